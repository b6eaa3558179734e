// msa_sort.hip -- LSD radix sort of the ranking entries, for large tables.
//
// Replaces qsort(entries, ..., entry_compare_desc) (parallel_spotify.c:178-188,
// 334, 1036, 1039) for tables of millions of distinct keys (configs[4]).  The
// entries' sort key is (K2 = ~count, K1 = key bytes 0..7, K0 = key bytes 8..15,
// big-endian) ascending, with the entry index as the value; runs of keys equal
// in all 24 bytes are ordered by k_tie_fixup afterwards, as for the merge sort
// (msa_post.hip) that small tables keep using.
//
// Design:
//   * one reduction finds the bits that differ anywhere in each key word:
//     8-bit digits that are the same in every entry are skipped (counts of a
//     high-cardinality table are small, so most bytes of K2 never vary);
//   * the words are sorted least significant first, each pass moving only
//     the current word and the entry index (12 B per entry, not the 28 B of
//     the whole key): the next word is gathered through the index once;
//   * a pass = per-tile digit histograms (4096 entries per workgroup) -> one
//     exclusive scan of the digit-major histogram matrix (= every tile's
//     output base per digit) -> a stable scatter: wave ballots split the
//     tile's entries by digit (8 ballots per 64 entries), the tile is staged
//     sorted in LDS, and each digit's run is written out contiguously.
#include "msa_internal.h"

#include <algorithm>

hipError_t msa_exclusive_scan(const u64 *in, u64 n, u64 *out, u64 *bsum_scratch, u64 *total, hipStream_t s);

namespace {

#define RX_T 256
#define RX_PER 16
#define RX_TILE (RX_T * RX_PER)
#define RX_W (RX_T / 64)

__device__ __forceinline__ u64 wave_or64(u64 v) {
    for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o);
    return v;
}

// bits that differ from entry 0's, per key word (vary[0] = K0, [1] = K1, [2] = K2)
__global__ __launch_bounds__(256) void k_rx_vary(const u64 *__restrict__ K2, const u64 *__restrict__ K1,
                                                 const u64 *__restrict__ K0, u64 n, u64 *__restrict__ vary) {
    const u64 f2 = K2[0], f1 = K1[0], f0 = K0[0];
    u64 v2 = 0, v1 = 0, v0 = 0;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        v2 |= K2[i] ^ f2;
        v1 |= K1[i] ^ f1;
        v0 |= K0[i] ^ f0;
    }
    v2 = wave_or64(v2);
    v1 = wave_or64(v1);
    v0 = wave_or64(v0);
    if (lane_id() == 0) {
        if (v0) atomicOr((unsigned long long *)&vary[0], (unsigned long long)v0);
        if (v1) atomicOr((unsigned long long *)&vary[1], (unsigned long long)v1);
        if (v2) atomicOr((unsigned long long *)&vary[2], (unsigned long long)v2);
    }
}

// ---- one-sweep passes: the digit histograms of every varying byte position
// are counted once up front (they do not depend on the order), so a pass is
// ONE kernel: tiles take tickets in order, rank their entries by digit within
// each wave (ballot multi-split + per-wave running counts in LDS), publish
// their per-digit counts and look back over earlier tiles' published counts
// (decoupled look-back, one digit per thread) for their global offsets.
#ifndef OS_T
#define OS_T 512
#endif
#ifndef OS_PER
#define OS_PER 16
#endif
#define OS_TILE (OS_T * OS_PER)
#define OS_W (OS_T / 64)
#ifndef GH_FLY
#define GH_FLY 4
#endif
#define OS_POS 24               // byte positions: K0 bytes 0..7, K1, K2
#ifndef OS_LB
#define OS_LB 1  // statuses per look-back round trip (8: configs[4] 28.5 -> 29.4 ms/step, the passes slower)
#endif
#define OS_SPIN_LIMIT (1u << 24)  // polls before a look-back gives up (error, never a hang)

// part[block][pos][digit] = entries of the block's stride with that digit at pos
__global__ __launch_bounds__(256) void k_os_ghist(const u64 *__restrict__ K0, const u64 *__restrict__ K1,
                                                  const u64 *__restrict__ K2, u64 n, u32 pmask,
                                                  u32 *__restrict__ part) {
    __shared__ u32 h[OS_POS * 256];
    const u32 t = threadIdx.x;
    for (u32 k = t; k < OS_POS * 256; k += 256) h[k] = 0;
    __syncthreads();
    // GH_FLY entries per thread per round, their loads issued first: one
    // entry per round left every wave waiting on its loads (8 waves per CU,
    // ~100 rounds each: 1.1 ms for configs[4]'s 50 M word entries)
    const u64 stride = (u64)gridDim.x * 256;
    for (u64 i0 = (u64)blockIdx.x * 256 + t; i0 < n; i0 += GH_FLY * stride) {
        u64 w[GH_FLY][3];
#pragma unroll
        for (u32 q = 0; q < GH_FLY; ++q) {
            const u64 i = i0 + q * stride;
            const bool ok = i < n;
            w[q][0] = ok && (pmask & 0xFFu) ? K0[i] : 0;
            w[q][1] = ok && (pmask & 0xFF00u) ? K1[i] : 0;
            w[q][2] = ok && (pmask & 0xFF0000u) ? K2[i] : 0;
        }
#pragma unroll
        for (u32 q = 0; q < GH_FLY; ++q) {
            if (i0 + q * stride >= n) break;
            const u64 act = __ballot(1);
#pragma unroll
            for (u32 p = 0; p < OS_POS; ++p) {
                if (!((pmask >> p) & 1u)) continue;
                const u32 d = (u32)(w[q][p >> 3] >> (8 * (p & 7))) & 0xFFu;
                // a digit the whole wave shares (zero padding of short keys, the
                // high bytes of small counts): one add instead of a 64-way conflict
                const u32 d0 = __builtin_amdgcn_readfirstlane(d);
                if (__ballot(d == d0) == act) {
                    if (mbcnt(act) == 0) atomicAdd(&h[p * 256 + d0], (u32)__popcll(act));
                } else {
                    atomicAdd(&h[p * 256 + d], 1u);
                }
            }
        }
    }
    __syncthreads();
    for (u32 k = t; k < OS_POS * 256; k += 256) part[(u64)blockIdx.x * (OS_POS * 256) + k] = h[k];
}

// gstart[pos][d] = entries whose digit at pos is below d (one block per
// varying position; four threads per digit sum the workgroup histograms)
#define GS_T 1024
__global__ __launch_bounds__(GS_T) void k_os_gscan(const u32 *__restrict__ part, u32 nparts, u32 pmask,
                                                   u64 *__restrict__ gstart) {
    __shared__ u32 c4[GS_T / 256][256];
    __shared__ u64 c[256];
    const u32 t = threadIdx.x, d = t & 255u, q = t >> 8, p = blockIdx.x;
    if (!((pmask >> p) & 1u)) return;  // a byte no pass sorts by
    u32 s = 0;
#pragma unroll 8
    for (u32 b = q; b < nparts; b += GS_T / 256) s += part[(u64)b * (OS_POS * 256) + p * 256 + d];
    c4[q][d] = s;
    __syncthreads();
    if (t < 256) {
        u64 tot = 0;
        for (u32 k = 0; k < GS_T / 256; ++k) tot += c4[k][t];
        c[t] = tot;
    }
    __syncthreads();
    if (t < 256) {
        u64 e = 0;
        for (u32 k = 0; k < t; ++k) e += c[k];
        gstart[p * 256 + t] = e;
    }
}

__device__ __forceinline__ u64 os_pack(u32 epoch, u32 incl, u32 v) {
    return ((u64)(epoch * 2u + incl) << 32) | v;
}

// One stable pass by the digit at `shift`.  status: [tile][digit] words
// (epoch, inclusive?, count), zeroed once per sort; epoch = pass number + 1.
__global__ __launch_bounds__(OS_T) void k_os_pass(const u64 *__restrict__ W, const u32 *__restrict__ V, u64 n,
                                                  u32 shift, const u64 *__restrict__ gstart,
                                                  u64 *__restrict__ status, u32 *__restrict__ ticket, u32 epoch,
                                                  u32 *__restrict__ err, u64 *__restrict__ Wo,
                                                  u32 *__restrict__ Vo) {
    __shared__ u64 sbuf[OS_TILE];
    __shared__ u32 wcnt[OS_W][256];
    __shared__ u32 lstart[256], wsum[4], stile;
    __shared__ u64 gbase[256];
    const u32 t = threadIdx.x, lane = lane_id(), w = t >> 6;
    for (u32 k = t; k < OS_W * 256; k += OS_T) (&wcnt[0][0])[k] = 0;
    if (t == 0) stile = atomicAdd(ticket, 1u);
    __syncthreads();
    const u32 tile = stile;
    const u64 tbase = (u64)tile * OS_TILE;
    const u64 base = tbase + (u64)w * (OS_PER * 64);
    u64 kw[OS_PER];
    u32 kv[OS_PER], lr[OS_PER];
#pragma unroll
    for (u32 j = 0; j < OS_PER; ++j) {
        const u64 e = base + (u64)j * 64 + lane;
        kw[j] = e < n ? W[e] : 0;
        kv[j] = e < n ? V[e] : 0;
    }
    // rank within the wave: lanes of a round with the same digit (8 ballots),
    // after the wave's earlier rounds (running count per digit in LDS; a wave's
    // LDS reads and writes execute in order)
#pragma unroll
    for (u32 j = 0; j < OS_PER; ++j) {
        const bool ok = base + (u64)j * 64 + lane < n;
        const u32 d = (u32)(kw[j] >> shift) & 0xFFu;
        u64 M = __ballot(ok);
#pragma unroll
        for (u32 b = 0; b < 8; ++b) {
            const u64 B = __ballot((d >> b) & 1u);
            M &= ((d >> b) & 1u) ? B : ~B;
        }
        const u32 r = mbcnt(M);
        const u32 pre = ok ? wcnt[w][d] : 0u;
        lr[j] = pre + r;
        if (ok && r == 0) wcnt[w][d] = pre + (u32)__popcll(M);
    }
    __syncthreads();
    u32 h = 0, pre = 0;
    if (t < 256) {
        for (u32 k = 0; k < OS_W; ++k) {  // per digit: wave offsets within the tile
            const u32 c = wcnt[k][t];
            wcnt[k][t] = h;
            h += c;
        }
        u64 *st = status + (u64)tile * 256 + t;
        u64 excl = 0;
        if (tile == 0) {
            __hip_atomic_store(st, os_pack(epoch, 1, h), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_store(st, os_pack(epoch, 0, h), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // look back OS_LB tiles per round trip (their statuses loaded
            // together; measured: more than one per trip slowed the passes)
            long long q = (long long)tile - 1;
            u32 spins = 0;
            bool done = false;
            while (!done) {
                u64 sv[OS_LB];
#pragma unroll
                for (u32 k = 0; k < OS_LB; ++k)
                    sv[k] = q - (long long)k >= 0 ? __hip_atomic_load(status + (u64)(q - (long long)k) * 256 + t, __ATOMIC_RELAXED,
                                                                __HIP_MEMORY_SCOPE_AGENT)
                                            : 0ull;
                u32 k = 0;
                for (; k < OS_LB; ++k) {
                    const u32 hi = (u32)(sv[k] >> 32);
                    if ((hi >> 1) != epoch) break;  // not published yet in this pass: reload from here
                    excl += (u32)sv[k];
                    if ((hi & 1u) || q - (long long)k == 0) {
                        done = true;
                        break;
                    }
                }
                if (done) break;
                q -= (long long)k;
                if (k == 0) {
                    if (++spins > OS_SPIN_LIMIT) {
                        atomicOr(err, 1u);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            __hip_atomic_store(st, os_pack(epoch, 1, (u32)(excl + h)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        gbase[t] = gstart[t] + excl;
        u32 tot;
        pre = wave_prefix<14>(h, tot);
        if (lane == 0) wsum[w] = tot;
    }
    __syncthreads();
    if (t < 256) {
        u32 add = 0;
        for (u32 k = 0; k < w; ++k) add += wsum[k];
        lstart[t] = pre + add;
    }
    __syncthreads();
#pragma unroll
    for (u32 j = 0; j < OS_PER; ++j) {
        if (base + (u64)j * 64 + lane < n) {
            const u32 d = (u32)(kw[j] >> shift) & 0xFFu;
            lr[j] += lstart[d] + wcnt[w][d];
            sbuf[lr[j]] = kw[j];
        }
    }
    __syncthreads();
    const u32 cnt = (u32)min((u64)OS_TILE, n - tbase);
    u32 g[OS_PER];
#pragma unroll
    for (u32 k = 0; k < OS_PER; ++k) {
        const u32 i = t + k * OS_T;
        if (i < cnt) {
            const u64 x = sbuf[i];
            const u32 d = (u32)(x >> shift) & 0xFFu;
            g[k] = (u32)(gbase[d] + (i - lstart[d]));
            Wo[g[k]] = x;
        }
    }
    __syncthreads();
    u32 *sv = reinterpret_cast<u32 *>(sbuf);
#pragma unroll
    for (u32 j = 0; j < OS_PER; ++j)
        if (base + (u64)j * 64 + lane < n) sv[lr[j]] = kv[j];
    __syncthreads();
#pragma unroll
    for (u32 k = 0; k < OS_PER; ++k) {
        const u32 i = t + k * OS_T;
        if (i < cnt) Vo[g[k]] = sv[i];
    }
}

// the next key word in the current order
__global__ void k_rx_gather(const u64 *__restrict__ src, const u32 *__restrict__ V, u64 n, u64 *__restrict__ out) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = src[V[i]];
}

// the sorted entries; word `wsel` (0 = K0 .. 2 = K2; 3 = none) is already in
// order in Ws (the last sorted word), the others are gathered through V
// kmode bit 0: keys hold no zero byte (words), so a key whose byte 7 is zero ended
// before byte 8 and its K0 is zero -- not gathered (most words are short)
// kmode bit 1: Ws holds composite keys (msa_radix_sort_comp) with the gid in
// the top kmode >> 4 bytes: a key whose last covered byte is zero ended
// there, so its K1 is the composite key shifted up and its K0 zero -- not
// gathered at all (short words: a third of configs[4]'s entries)
__global__ void k_rx_final(const u64 *__restrict__ K2, const u64 *__restrict__ K1, const u64 *__restrict__ K0,
                           const u32 *__restrict__ V, u64 n, const u64 *__restrict__ Ws, u32 wsel, u32 kmode,
                           u64 *__restrict__ O2, u64 *__restrict__ O1, u64 *__restrict__ O0, u32 *__restrict__ OV) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u32 v = V[i];
    const u64 w2 = wsel == 2 ? Ws[i] : K2[v];
    if (O2) O2[i] = w2;  // null: the caller keeps Ws as the sorted K2 plane
    // (K1 and K0 loaded together for every longer key: 1.84 vs 1.61-1.64 ms)
    if ((kmode & 2u) && wsel == 2 && !(w2 & 0xFFu)) {
        O1[i] = w2 << (8 * (kmode >> 4));
        O0[i] = 0;
    } else {
        const u64 k1 = wsel == 1 ? Ws[i] : K1[v];
        O1[i] = k1;
        O0[i] = wsel == 0 ? Ws[i] : (((kmode & 1u) && !(k1 & 0xFFu)) ? 0ull : K0[v]);
    }
    if (OV) OV[i] = v;  // null: the caller keeps V as the sorted values
}

inline dim3 g1(u64 n, u32 t = 256) { return dim3((u32)((n + t - 1) / t)); }
inline u64 os_tiles(u64 n) { return (n + OS_TILE - 1) / OS_TILE; }
inline u32 os_parts(u64 n) { return (u32)std::max<u64>(1, std::min<u64>(512, (n + 4095) / 4096)); }

}  // namespace

// vary (64 B) | tickets + error word (256 B) | gstart | part | status
u64 msa_radix_scratch_bytes(u64 n) {
    return 64 + 256 + (u64)OS_POS * 256 * 8 + (u64)os_parts(n) * OS_POS * 256 * 4 + os_tiles(n) * 256 * 8 + 64;
}

// Sorts set 0 (K2, K1, K0, V: the entries, V[0][i] = i) ascending; the result
// lands in set 1 or 2 (*which).  Sets 1 and 2 are scratch, as for
// msa_launch_sort.  `scratch` holds msa_radix_scratch_bytes(n) bytes.
hipError_t msa_radix_sort(u64 *const K2[3], u64 *const K1[3], u64 *const K0[3], u32 *const V[3], u64 n, int *which,
                          u8 *scratch, hipStream_t s, const u64 *vary_pre, bool sort_k0, const u64 *hv_host,
                          u32 kmode, u64 **ws_keep, u32 **v_keep) {
    if (ws_keep) *ws_keep = nullptr;
    if (v_keep) *v_keep = nullptr;
    *which = 1;
    if (!n) return hipSuccess;
    if (n >= (1ull << 32)) return hipErrorInvalidValue;  // u32 indices and counts
    const u64 ntiles = os_tiles(n);
    const u32 nparts = os_parts(n);
    u64 *vary = reinterpret_cast<u64 *>(scratch);
    u32 *tickets = reinterpret_cast<u32 *>(scratch + 64), *err = tickets + 63;
    u64 *gstart = reinterpret_cast<u64 *>(scratch + 64 + 256);
    u32 *part = reinterpret_cast<u32 *>(gstart + OS_POS * 256);
    u64 *status = reinterpret_cast<u64 *>(part + (u64)nparts * OS_POS * 256);
    hipError_t e;
    if ((e = hipMemsetAsync(scratch, 0, 64 + 256, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(status, 0, ntiles * 256 * 8, s)) != hipSuccess) return e;
    u64 hv[6];
    if (hv_host) {  // the varying bits of each word, known to the caller
        for (int w = 0; w < 3; ++w) hv[w] = hv_host[w];
    } else if (vary_pre) {  // the planes' OR / AND from the entries' builder
        if ((e = hipMemcpyAsync(hv, vary_pre, sizeof hv, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        for (int w = 0; w < 3; ++w) hv[w] &= ~hv[3 + w];
    } else {
        hipLaunchKernelGGL(k_rx_vary, dim3((u32)std::min<u64>(1024, (n + 255) / 256)), dim3(256), 0, s, K2[0], K1[0],
                           K0[0], n, vary);
        if ((e = hipMemcpyAsync(hv, vary, 3 * sizeof(u64), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    }
    if (!sort_k0) hv[0] = 0;  // K0's bytes are left to the tie refinement (refine_ties)
    u32 pmask = 0;
    for (int wi = 0; wi < 3; ++wi)
        for (u32 b = 0; b < 8; ++b)
            if ((hv[wi] >> (8 * b)) & 0xFFull) pmask |= 1u << (wi * 8 + b);
    if (pmask) {
        hipLaunchKernelGGL(k_os_ghist, dim3(nparts), dim3(256), 0, s, K0[0], K1[0], K2[0], n, pmask, part);
        hipLaunchKernelGGL(k_os_gscan, dim3(OS_POS), dim3(GS_T), 0, s, (const u32 *)part, nparts, pmask, gstart);
    }

    const u64 *orig[3] = {K0[0], K1[0], K2[0]};  // least significant word first
    u64 *Wb[3] = {nullptr, K0[1], K0[2]};
    const u64 *Wp = nullptr;
    int vloc = 0;
    bool any = false;
    u32 pass = 0, wsel = 3;
    for (int wi = 0; wi < 3; ++wi) {
        if (!hv[wi]) continue;
        if (!any) {
            Wp = orig[wi];
        } else {  // the new word in the current order, into the free W buffer
            u64 *dst = Wb[vloc];
            hipLaunchKernelGGL(k_rx_gather, g1(n), dim3(256), 0, s, orig[wi], (const u32 *)V[vloc], n, dst);
            Wp = dst;
        }
        any = true;
        wsel = (u32)wi;
        for (u32 b = 0; b < 8; ++b) {
            if (!((hv[wi] >> (8 * b)) & 0xFFull)) continue;  // the same byte in every entry
            const int dst = (vloc == 1 || Wp == Wb[1]) ? 2 : 1;
            hipLaunchKernelGGL(k_os_pass, dim3((u32)ntiles), dim3(OS_T), 0, s, Wp, (const u32 *)V[vloc], n, 8 * b,
                               (const u64 *)(gstart + (wi * 8 + b) * 256), status, tickets + pass, pass + 1, err,
                               Wb[dst], V[dst]);
            ++pass;
            vloc = dst;
            Wp = Wb[dst];
        }
    }
    const int o = vloc == 1 ? 2 : 1;
    // Wp: the last sorted word in order (unless it was gathered into set o's K0 buffer)
    if (wsel < 3 && Wp == K0[o]) wsel = 3;
    // ws_keep: the sorted K2 words stay where the last pass left them (the
    // caller takes that buffer as set o's K2 plane) instead of being copied
    // (v_keep: likewise the sorted values, when a pass wrote them)
    const bool keep = ws_keep && wsel == 2;
    if (keep) *ws_keep = const_cast<u64 *>(Wp);
    const bool vk = v_keep && vloc != 0;
    if (vk) *v_keep = V[vloc];
    hipLaunchKernelGGL(k_rx_final, g1(n), dim3(256), 0, s, K2[0], K1[0], K0[0], (const u32 *)V[vloc], n, Wp, wsel,
                       kmode, keep ? nullptr : K2[o], K1[o], K0[o], vk ? nullptr : V[o]);
    *which = o;
    if ((e = hipGetLastError()) != hipSuccess) return e;
    u32 herr = 0;  // a look-back that gave up (never expected: tiles take tickets in order)
    if ((e = hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    return herr ? hipErrorLaunchFailure : hipSuccess;
}

// ---------------------------------------------------------------------------
// Words' composite sort key.  The ranking order is (count descending, key
// ascending); counts take few distinct values (at most ~sqrt(2 * total
// words): ~15 K for configs[4]'s 107 M words), so each count is replaced by
// its dense rank among the distinct counts (gid, 0 = the largest count) in
// the top 1-2 bytes of ONE 64-bit word whose other bytes are the key's first
// bytes: C = gid << (64 - 8 gB) | K1 >> 8 gB.  Sorting C alone (8 passes at
// most) replaces the passes over the count's varying bytes (3 for configs[4])
// and the gather of the second word between the two words' passes; entries
// equal in C are ordered by the tie refinement from key byte 8 - gB on.
#define CS_SLOTS (1u << 18)  // distinct-count set (open addressing, <= 25 % full)
#define CS_MAXD 65536u       // distinct counts the composite key takes (2-byte gid)
#define CS_PROBE 256u        // probes before the set counts as full
namespace {
__device__ __forceinline__ u32 cs_hash(u64 v) {
    v ^= v >> 33;
    v *= 0xff51afd7ed558ccdull;
    v ^= v >> 29;
    return (u32)v & (CS_SLOTS - 1);
}
struct CsBufs {
    u32 *meta;  // [0] distinct counts inserted, [1] listed, [2] a probe run gave up
    u64 *set;   // count + 1 per used slot
    u32 *rk;    // listed count -> gid (summed over k_cset_rank's tiles)
    u32 *gidv;  // slot -> gid
    u32 *list;  // used slots
    u64 *gcnt;  // gid -> count
};
inline CsBufs cs_bufs(u8 *p) {
    CsBufs b;
    b.meta = reinterpret_cast<u32 *>(p);
    b.set = reinterpret_cast<u64 *>(p + 64);
    b.rk = reinterpret_cast<u32 *>(b.set + CS_SLOTS);
    b.gidv = b.rk + CS_MAXD;
    b.list = b.gidv + CS_SLOTS;
    b.gcnt = reinterpret_cast<u64 *>(b.list + CS_MAXD);
    return b;
}
#define CS_FLY 4
#define CS_LSLOTS 2048u  // per-workgroup set in LDS
// v into the device set: compare-and-swap first (its returned value is the
// slot's word at the memory side; a plain load may read a stale zero from
// this CU's L1 for the whole kernel -- every later lane then CASes the same
// hot slot: 4.3 ms for 50 M entries)
__device__ __forceinline__ void cs_put(const CsBufs &b, u64 v) {
    u32 h = cs_hash(v);
    for (u32 p = 0; p < CS_PROBE; ++p) {
        const u64 old = atomicCAS((unsigned long long *)&b.set[h], 0ull, (unsigned long long)v);
        if (old == 0) {
            atomicAdd(&b.meta[0], 1u);
            return;
        }
        if (old == v) return;
        h = (h + 1) & (CS_SLOTS - 1);
    }
    atomicOr(&b.meta[2], 1u);  // far too many distinct counts: the caller falls back
}
// Each workgroup collects its entries' distinct counts in LDS, then puts each
// into the device set once.
__global__ __launch_bounds__(256) void k_cset_insert(const u64 *__restrict__ K2, u64 n, CsBufs b) {
    __shared__ u64 ls[CS_LSLOTS];
    for (u32 k = threadIdx.x; k < CS_LSLOTS; k += 256) ls[k] = 0;
    __syncthreads();
    const u64 stride = (u64)gridDim.x * 256;
    for (u64 i0 = (u64)blockIdx.x * 256 + threadIdx.x; i0 < n; i0 += CS_FLY * stride) {
        u64 v[CS_FLY];
#pragma unroll
        for (u32 q = 0; q < CS_FLY; ++q) {
            const u64 i = i0 + q * stride;
            v[q] = i < n ? ~K2[i] + 1 : 0;  // count + 1: never 0
        }
#pragma unroll
        for (u32 q = 0; q < CS_FLY; ++q) {
            if (!v[q]) continue;
            // a count the whole wave shares (count 1 of a high-cardinality
            // table): one lane inserts it
            const u64 v0 = __builtin_amdgcn_readfirstlane(v[q]);
            if (__ballot(v[q] == v0) == __ballot(1) && mbcnt(__ballot(1)) != 0) continue;
            u32 h = cs_hash(v[q]) & (CS_LSLOTS - 1);
            u32 p = 0;
            for (; p < 32; ++p) {
                const u64 old = atomicCAS((unsigned long long *)&ls[h], 0ull, (unsigned long long)v[q]);
                if (old == 0 || old == v[q]) break;
                h = (h + 1) & (CS_LSLOTS - 1);
            }
            if (p == 32) cs_put(b, v[q]);  // the workgroup's set is crowded
        }
    }
    __syncthreads();
    for (u32 k = threadIdx.x; k < CS_LSLOTS; k += 256)
        if (ls[k]) cs_put(b, ls[k]);
}
// the used slots, listed (one claim per workgroup: a claim per wave on the
// one counter serialised, 150 us)
__global__ __launch_bounds__(1024) void k_cset_list(CsBufs b) {
    __shared__ u32 wc[16], wb[16], gb;
    const u32 t = threadIdx.x, w = t >> 6, sl = blockIdx.x * 1024 + t;
    const bool used = b.set[sl] != 0;
    const u64 M = __ballot(used);
    if (lane_id() == 0) wc[w] = (u32)__popcll(M);
    __syncthreads();
    if (t == 0) {
        u32 tot = 0;
        for (u32 k = 0; k < 16; ++k) {
            wb[k] = tot;
            tot += wc[k];
        }
        gb = tot ? atomicAdd(&b.meta[1], tot) : 0u;
    }
    __syncthreads();
    const u32 at = gb + wb[w] + mbcnt(M);
    if (used && at < CS_MAXD) b.list[at] = sl;
}
// gid of listed count i = listed counts larger than it: workgroup (x, y)
// counts, for its 256 listed counts, the larger ones among listed counts
// [y CR_TILE, (y + 1) CR_TILE) (a grid over both, not one thread looping over
// all of them: 330 us for ~25 K distinct counts); k_cset_fin stores the gids
#define CR_TILE 2048
__global__ __launch_bounds__(256) void k_cset_rank(CsBufs b) {
    __shared__ u64 tile[CR_TILE];
    const u32 m = min(b.meta[1], CS_MAXD);
    if (b.meta[0] > CS_MAXD || b.meta[2]) return;
    const u32 j0 = blockIdx.y * CR_TILE;
    if (blockIdx.x * 256 >= m || j0 >= m) return;  // whole workgroup
    const u32 i = blockIdx.x * 256 + threadIdx.x;
    const u32 tn = min(CR_TILE, m - j0);
    for (u32 k = threadIdx.x; k < tn; k += 256) tile[k] = b.set[b.list[j0 + k]];
    const u64 v = i < m ? b.set[b.list[i]] : ~0ull;
    __syncthreads();
    u32 r = 0;
    for (u32 k = 0; k < tn; ++k) r += tile[k] > v;
    if (i < m && r) atomicAdd(&b.rk[i], r);
}
__global__ __launch_bounds__(256) void k_cset_fin(CsBufs b) {
    const u32 m = min(b.meta[1], CS_MAXD);
    if (b.meta[0] > CS_MAXD || b.meta[2]) return;
    const u32 i = blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    const u32 sl = b.list[i], r = b.rk[i];
    b.gidv[sl] = r;
    b.gcnt[r] = b.set[sl] - 1;
}
__device__ __forceinline__ u32 cs_gid(const CsBufs &b, u64 v) {
    u32 h = cs_hash(v);
    for (u32 p = 0; p < CS_PROBE; ++p) {
        if (b.set[h] == v) return b.gidv[h];
        h = (h + 1) & (CS_SLOTS - 1);
    }
    return 0;  // never: every count was inserted
}
__global__ __launch_bounds__(256) void k_comp_build(const u64 *__restrict__ K2, const u64 *__restrict__ K1, u64 n,
                                                    CsBufs b, u32 gB, u64 *__restrict__ C) {
    const u64 stride = (u64)gridDim.x * 256;
    for (u64 i0 = (u64)blockIdx.x * 256 + threadIdx.x; i0 < n; i0 += CS_FLY * stride) {
        u64 v[CS_FLY], k1[CS_FLY];
#pragma unroll
        for (u32 q = 0; q < CS_FLY; ++q) {
            const u64 i = i0 + q * stride;
            v[q] = i < n ? ~K2[i] + 1 : 0;
            k1[q] = i < n ? K1[i] : 0;
        }
#pragma unroll
        for (u32 q = 0; q < CS_FLY; ++q) {
            const u64 i = i0 + q * stride;
            if (i >= n) break;
            if (!gB) {
                C[i] = k1[q];
                continue;
            }
            const u32 g = cs_gid(b, v[q]);
            C[i] = ((u64)g << (64 - 8 * gB)) | (k1[q] >> (8 * gB));
        }
    }
}
// sorted C -> ~count, in place
__global__ void k_comp_k2(u64 *__restrict__ P, u64 n, const u64 *__restrict__ gcnt, u32 gB) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    P[i] = ~gcnt[gB ? (u32)(P[i] >> (64 - 8 * gB)) : 0u];
}
}  // namespace

u64 msa_comp_scratch_bytes() { return 64 + (u64)CS_SLOTS * 12 + (u64)CS_MAXD * 16 + 64; }

// The words' sort by the composite key (above).  *gB_out = gid bytes (key
// bytes 0 .. 7 - gB are sorted), or ~0u when the table's counts take more
// than CS_MAXD distinct values (nothing sorted: the caller sorts K2/K1).
// vary_pre: the planes' OR / AND from k_word_entries (device, 6 words).
// C: n words of scratch; after the sort set *which's K2 plane holds the sorted
// composite keys (msa_comp_finish turns them into ~count).
hipError_t msa_radix_sort_comp(u64 *const K2[3], u64 *const K1[3], u64 *const K0[3], u32 *const V[3], u64 n,
                               int *which, u8 *scratch, hipStream_t s, const u64 *vary_pre, u64 *C, u8 *cs,
                               u32 *gB_out, u64 **ws_keep, u32 **v_keep) {
    *gB_out = ~0u;
    *ws_keep = nullptr;
    *v_keep = nullptr;
    if (!n || n >= (1ull << 32)) return hipSuccess;
    const CsBufs b = cs_bufs(cs);
    hipError_t e;
    if ((e = hipMemsetAsync(cs, 0, 64 + (u64)CS_SLOTS * 8 + (u64)CS_MAXD * 4, s)) != hipSuccess) return e;  // meta, set, rk
    const u32 g = (u32)std::min<u64>(2048, (n + 1023) / 1024);
    hipLaunchKernelGGL(k_cset_insert, dim3(g), dim3(256), 0, s, (const u64 *)K2[0], n, b);
    hipLaunchKernelGGL(k_cset_list, dim3(CS_SLOTS / 1024), dim3(1024), 0, s, b);
    hipLaunchKernelGGL(k_cset_rank, dim3(CS_MAXD / 256, CS_MAXD / CR_TILE), dim3(256), 0, s, b);
    hipLaunchKernelGGL(k_cset_fin, dim3(CS_MAXD / 256), dim3(256), 0, s, b);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    u64 hv[8];
    u32 meta[3];
    if ((e = hipMemcpyAsync(hv, vary_pre, 6 * 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(meta, b.meta, 12, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    const u32 m = meta[0];
    if (m == 0 || m > CS_MAXD || meta[1] != m || meta[2]) return hipSuccess;
    const u32 gB = m == 1 ? 0 : (m <= 256 ? 1 : 2);
    u64 vk1 = hv[1] & ~hv[4];  // K1's varying bits
    u64 vc = gB ? vk1 >> (8 * gB) : vk1;
    if (gB) {
        u64 gm = m - 1;  // gids 0 .. m-1: the bits below m-1's top bit may vary
        gm |= gm >> 1; gm |= gm >> 2; gm |= gm >> 4; gm |= gm >> 8; gm |= gm >> 16;
        vc |= gm << (64 - 8 * gB);
    }
    hipLaunchKernelGGL(k_comp_build, dim3(g), dim3(256), 0, s, (const u64 *)K2[0], (const u64 *)K1[0], n, b, gB, C);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    u64 *const Kc[3] = {C, K2[1], K2[2]};
    const u64 hvc[3] = {0, 0, vc};
    if ((e = msa_radix_sort(Kc, K1, K0, V, n, which, scratch, s, nullptr, false, hvc, 1u | 2u | (gB << 4), ws_keep, v_keep)) != hipSuccess)
        return e;
    *gB_out = gB;
    return hipSuccess;
}
hipError_t msa_comp_finish(u64 *P, u64 n, const u8 *cs, u32 gB, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_comp_k2, g1(n), dim3(256), 0, s, P, n, (const u64 *)cs_bufs(const_cast<u8 *>(cs)).gcnt, gB);
    return hipGetLastError();
}
