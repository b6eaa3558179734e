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

// th[d * ntiles + tile] = entries of the tile whose digit is d
__global__ __launch_bounds__(RX_T) void k_rx_hist(const u64 *__restrict__ W, u64 n, u32 shift, u32 ntiles,
                                                  u64 *__restrict__ th) {
    __shared__ u32 h[256];
    const u32 t = threadIdx.x;
    h[t] = 0;
    __syncthreads();
    const u64 base = (u64)blockIdx.x * RX_TILE;
#pragma unroll 4
    for (u32 j = 0; j < RX_PER; ++j) {
        const u64 e = base + (u64)j * RX_T + t;
        if (e < n) atomicAdd(&h[(u32)(W[e] >> shift) & 0xFFu], 1u);
    }
    __syncthreads();
    th[(u64)t * ntiles + blockIdx.x] = h[t];
}

// Stable scatter of one tile by the digit at `shift`; toff = the scanned th.
__global__ __launch_bounds__(RX_T) void k_rx_scatter(const u64 *__restrict__ W, const u32 *__restrict__ V, u64 n,
                                                     u32 shift, u32 ntiles, const u64 *__restrict__ toff,
                                                     u64 *__restrict__ Wo, u32 *__restrict__ Vo) {
    __shared__ u64 sW[RX_TILE];
    __shared__ u32 sV[RX_TILE];
    __shared__ u32 h[256], lstart[256], run[256], wsum[RX_W];
    __shared__ u32 wcnt[RX_W][256], wpre[RX_W][256];
    const u32 t = threadIdx.x, lane = lane_id(), w = t >> 6;
    const u64 lt = (1ull << lane) - 1ull;
    const u64 base = (u64)blockIdx.x * RX_TILE;
    h[t] = 0;
    run[t] = 0;
    for (u32 k = 0; k < RX_W; ++k) wcnt[k][t] = 0;
    __syncthreads();
    u64 kw[RX_PER];
    u32 kv[RX_PER];
#pragma unroll
    for (u32 j = 0; j < RX_PER; ++j) {
        const u64 e = base + (u64)j * RX_T + t;
        kw[j] = e < n ? W[e] : 0;
        kv[j] = e < n ? V[e] : 0;
        if (e < n) atomicAdd(&h[(u32)(kw[j] >> shift) & 0xFFu], 1u);
    }
    __syncthreads();
    {  // lstart = exclusive scan of h (256 digits: 4 waves of 64)
        const u32 x = h[t];
        u32 tot;
        const u32 pre = wave_prefix<13>(x, tot);
        if (lane == 0) wsum[w] = tot;
        __syncthreads();
        u32 add = 0;
        for (u32 k = 0; k < w; ++k) add += wsum[k];
        lstart[t] = pre + add;
    }
    __syncthreads();
#pragma unroll
    for (u32 j = 0; j < RX_PER; ++j) {
        const u64 e = base + (u64)j * RX_T + t;
        const bool ok = e < n;
        const u32 d = (u32)(kw[j] >> shift) & 0xFFu;
        // lanes holding the same digit (multi-split by ballots)
        u64 M = __ballot(ok);
#pragma unroll
        for (u32 b = 0; b < 8; ++b) {
            const u64 B = __ballot((d >> b) & 1u);
            M &= ((d >> b) & 1u) ? B : ~B;
        }
        const u32 rank = (u32)__popcll(M & lt);
        if (ok && rank == 0) wcnt[w][d] = (u32)__popcll(M);
        __syncthreads();
        {  // per digit: earlier waves of this round, after earlier rounds
            u32 b0 = run[t];
            for (u32 k = 0; k < RX_W; ++k) {
                wpre[k][t] = b0;
                b0 += wcnt[k][t];
                wcnt[k][t] = 0;
            }
            run[t] = b0;
        }
        __syncthreads();
        if (ok) {
            const u32 pos = lstart[d] + wpre[w][d] + rank;
            sW[pos] = kw[j];
            sV[pos] = kv[j];
        }
    }
    __syncthreads();
    const u32 cnt = (u32)min((u64)RX_TILE, n - base);
    for (u32 i = t; i < cnt; i += RX_T) {
        const u64 x = sW[i];
        const u32 d = (u32)(x >> shift) & 0xFFu;
        const u64 g = toff[(u64)d * ntiles + blockIdx.x] + (i - lstart[d]);
        Wo[g] = x;
        Vo[g] = sV[i];
    }
}

// the next key word in the current order
__global__ void k_rx_gather(const u64 *__restrict__ src, const u32 *__restrict__ V, u64 n, u64 *__restrict__ out) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = src[V[i]];
}

__global__ void k_rx_final(const u64 *__restrict__ K2, const u64 *__restrict__ K1, const u64 *__restrict__ K0,
                           const u32 *__restrict__ V, u64 n, u64 *__restrict__ O2, u64 *__restrict__ O1,
                           u64 *__restrict__ O0, u32 *__restrict__ OV) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u32 v = V[i];
    O2[i] = K2[v];
    O1[i] = K1[v];
    O0[i] = K0[v];
    OV[i] = v;
}

inline dim3 g1(u64 n, u32 t = 256) { return dim3((u32)((n + t - 1) / t)); }
inline u64 rx_tiles(u64 n) { return (n + RX_TILE - 1) / RX_TILE; }

}  // namespace

u64 msa_radix_scratch_bytes(u64 n) {
    const u64 m = 256 * rx_tiles(n);
    return 64 + 2 * m * 8 + ((m + 1023) / 1024 + 1) * 8 + 64;
}

// Sorts set 0 (K2, K1, K0, V: the entries, V[0][i] = i) ascending; the result
// lands in set 1 or 2 (*which).  Sets 1 and 2 are scratch, as for
// msa_launch_sort.  `scratch` holds msa_radix_scratch_bytes(n) bytes.
hipError_t msa_radix_sort(u64 *const K2[3], u64 *const K1[3], u64 *const K0[3], u32 *const V[3], u64 n, int *which,
                          u8 *scratch, hipStream_t s) {
    *which = 1;
    if (!n) return hipSuccess;
    const u64 ntiles = rx_tiles(n), m = 256 * ntiles;
    u64 *vary = reinterpret_cast<u64 *>(scratch);
    u64 *th = vary + 8, *toff = th + m, *bsum = toff + m, *total = bsum + (m + 1023) / 1024 + 1;
    hipError_t e;
    if ((e = hipMemsetAsync(vary, 0, 64, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_rx_vary, dim3((u32)std::min<u64>(1024, (n + 255) / 256)), dim3(256), 0, s, K2[0], K1[0],
                       K0[0], n, vary);
    u64 hv[3];
    if ((e = hipMemcpyAsync(hv, vary, sizeof hv, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;

    const u64 *orig[3] = {K0[0], K1[0], K2[0]};  // least significant word first
    u64 *Wb[3] = {nullptr, K0[1], K0[2]};
    const u64 *Wp = nullptr;
    int vloc = 0;
    bool any = false;
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
        for (u32 b = 0; b < 8; ++b) {
            if (!((hv[wi] >> (8 * b)) & 0xFFull)) continue;  // the same byte in every entry
            const int dst = (vloc == 1 || Wp == Wb[1]) ? 2 : 1;
            hipLaunchKernelGGL(k_rx_hist, dim3((u32)ntiles), dim3(RX_T), 0, s, Wp, n, 8 * b, (u32)ntiles, th);
            if ((e = msa_exclusive_scan(th, m, toff, bsum, total, s)) != hipSuccess) return e;
            hipLaunchKernelGGL(k_rx_scatter, dim3((u32)ntiles), dim3(RX_T), 0, s, Wp, (const u32 *)V[vloc], n, 8 * b,
                               (u32)ntiles, (const u64 *)toff, Wb[dst], V[dst]);
            vloc = dst;
            Wp = Wb[dst];
        }
    }
    const int o = vloc == 1 ? 2 : 1;
    hipLaunchKernelGGL(k_rx_final, g1(n), dim3(256), 0, s, K2[0], K1[0], K0[0], (const u32 *)V[vloc], n, K2[o], K1[o],
                       K0[o], V[o]);
    *which = o;
    return hipGetLastError();
}
