// msa_k1.h -- the chunk transfer function of the CSV reader (K1), one 4 KiB
// block at a time, from the block's byte-class masks.  Shared by the
// stand-alone summary kernel (k_chunk_summary, msa_scan.hip: the artist column
// and CPU-free callers) and the folded split scan (k_scan_fold, msa_k3.hip).
//
// Follows the record reader of the reference (read_csv_record,
// parallel_spotify.c:549-633): a terminator is an unquoted '\r' or an unquoted
// '\n' not preceded by an unquoted '\r'; unquoted commas count the fields
// (parse_csv_line 258-304, saturated at 3); a NUL ends the C string.
#pragma once
#include "msa_internal.h"

// bit j = xor of bits < j (the quote parity before each byte)
__device__ __forceinline__ u64 k1_pxor_excl64(u64 q) {
    u64 x = q << 1;
    x ^= x << 1;
    x ^= x << 2;
    x ^= x << 4;
    x ^= x << 8;
    x ^= x << 16;
    x ^= x << 32;
    return x;
}

// lane l receives lane l+1's value (lane 63: 0) / lane l-1's (lane 0: 0):
// DPP wave shifts (VALU, a few cycles) instead of ds_bpermute (LDS latency in
// the block's dependency chain)
__device__ __forceinline__ u64 k1_from_next(u64 v) {
    const u32 lo = __builtin_amdgcn_update_dpp(0u, (u32)v, 0x130, 0xF, 0xF, false);
    const u32 hi = __builtin_amdgcn_update_dpp(0u, (u32)(v >> 32), 0x130, 0xF, 0xF, false);
    return ((u64)hi << 32) | lo;
}
__device__ __forceinline__ u64 k1_from_prev(u64 v) {
    const u32 lo = __builtin_amdgcn_update_dpp(0u, (u32)v, 0x138, 0xF, 0xF, false);
    const u32 hi = __builtin_amdgcn_update_dpp(0u, (u32)(v >> 32), 0x138, 0xF, 0xF, false);
    return ((u64)hi << 32) | lo;
}

// A chunk's function under both incoming quote parities (h = 0 / 1), built
// block by block.  Per lane: terminators seen (summed over the wave once per
// chunk); wave-uniform: the rest.
struct K1Acc {
    u32 par, first_nl, anyrare;
    u32 cr[2], ntl[2], cc[2], zz[2], lend[2];
};
__device__ __forceinline__ void k1_init(K1Acc &s) {
    s.par = s.first_nl = s.anyrare = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) s.cr[h] = s.ntl[h] = s.cc[h] = s.zz[h] = s.lend[h] = 0;
}

// One block: the lane's 64-byte masks (bytes past the chunk end cleared), the
// raw '\n' flag of the byte after the block (the '\r\n' swallow at lane 63),
// off = the block's offset in the chunk, lastb = the offset of its last valid
// byte in the block.
__device__ __forceinline__ void k1_block(K1Acc &s, u64 Q, u64 C, u64 NL, u64 CR, u64 Z, bool rare, u32 nb_nl,
                                         u32 off, u32 lastb) {
    const u32 lane = lane_id();
    s.anyrare |= rare ? 1u : 0u;
    if (off == 0) s.first_nl = (u32)(readlane64(NL, 0) & 1u);
    const u64 B = __ballot(__popcll(Q) & 1u);
    const u32 pin0 = s.par ^ (mbcnt(B) & 1u);
    const u64 inq0 = k1_pxor_excl64(Q) ^ (pin0 ? ~0ull : 0ull);
    s.par ^= (u32)__popcll(B) & 1u;
    const u64 dn = k1_from_next(NL);  // every lane active (whole-wave calls)
    const u64 nlnext = (NL >> 1) | ((u64)((lane == 63) ? nb_nl : (u32)(dn & 1u)) << 63);
    const int Lz = (int)(lastb >> 6);
    const u32 bz = lastb & 63u;
    const u64 Bz = __ballot(Z != 0);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const u64 inq = h ? ~inq0 : inq0;
        const u64 CRu = CR & ~inq, NLu = NL & ~inq, Cu = C & ~inq;
        const u64 up = k1_from_prev(CRu);
        const u64 pc0 = lane ? ((up >> 63) & 1u) : (u64)s.cr[h];
        const u64 TERM = CRu | (NLu & ~((CRu << 1) | pc0));
        const u32 nt = (u32)__popcll(TERM);
        s.ntl[h] += nt;
        const u32 cq = min((u32)__popcll(Cu), 3u);
        const u64 C1 = __ballot(cq >= 1u), C2 = __ballot(cq >= 2u), C3 = __ballot(cq >= 3u);
        const u64 Bh = __ballot(nt != 0);
        if (Bh) {
            const int jl = 63 - __clzll(Bh);
            const u64 A = (jl == 63) ? 0ull : (~0ull << (jl + 1));  // lanes after jl
            const u64 tj = readlane64(TERM, jl);
            const u32 lt_j = 63u - (u32)__clzll(tj);
            const u64 above = lt_j == 63 ? 0ull : (~0ull << (lt_j + 1));
            const u32 c_new = (u32)__popcll(readlane64(Cu, jl) & above) + (u32)__popcll(C1 & A) +
                              (u32)__popcll(C2 & A) + (u32)__popcll(C3 & A);
            s.cc[h] = min(c_new, 3u);
            s.zz[h] = ((readlane64(Z, jl) & above) != 0) | ((Bz & A) != 0);
            const u32 sw_j = (u32)(((readlane64(CRu, jl) & readlane64(nlnext, jl)) >> lt_j) & 1u);
            s.lend[h] = off + (u32)jl * 64u + lt_j + 1u + sw_j;
        } else {
            s.cc[h] = min(s.cc[h] + (u32)__popcll(C1) + (u32)__popcll(C2) + (u32)__popcll(C3), 3u);
            s.zz[h] |= (Bz != 0);
        }
        s.cr[h] = (u32)((readlane64(CRu, Lz) >> bz) & 1u);
    }
}

// The chunk's summary (wave-uniform; <= 16384 terminators a chunk: 15 bits)
__device__ __forceinline__ ChunkSum k1_finish(const K1Acc &s) {
    ChunkSum r;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        u32 tot = 0;
#pragma unroll
        for (int b = 0; b < 15; ++b) tot += (u32)__popcll(__ballot((s.ntl[h] >> b) & 1u)) << b;
        r.h[h] = tot | (s.cc[h] << 16) | (s.zz[h] << 18) | (s.cr[h] << 19) | (s.par << 20) | (s.first_nl << 21) |
                 (s.anyrare << 22);
        r.last_end[h] = s.lend[h];
    }
    return r;
}

// The 4 KiB block through LDS: loaded coalesced (instruction q: 1 KiB, lane l
// the 16 bytes at 1024 q + 16 l -- 16 lines of 64 B per instruction instead of
// 64 when every lane reads its own 64 contiguous bytes; those loads kept the
// texture data path ~82 % busy, profiles/r06_pmc_tok_explore.txt), written to
// the wave's LDS image and read back as lane l = bytes [64 l, 64 l + 64).
// 16-byte chunk c sits at c ^ ((c >> 4) & 3): the reads' 16-lane groups then
// hit 16 different slots of the 256-byte bank row (4-way conflicts without),
// and the writes' 8-lane groups stay on 8 different slots.
__device__ __forceinline__ u32 blk_swz(u32 c) { return c ^ ((c >> 4) & 3u); }
// (four named registers, not an array: an array the two prefetch sites
// assign was kept in scratch memory)
struct Blk4 {
    uint4 a, b, c, d;
};
__device__ __forceinline__ Blk4 blk_load_co(const u8 *p) {
    const u32 lane = lane_id();
    const uint4 *q = reinterpret_cast<const uint4 *>(p + 16 * lane);
    return Blk4{q[0], q[64], q[128], q[192]};
}
__device__ __forceinline__ void blk_transpose(uint4 *st, const Blk4 &r, uint4 (&o)[4]) {
    const u32 lane = lane_id();
    st[blk_swz(lane)] = r.a;
    st[blk_swz(64 + lane)] = r.b;
    st[blk_swz(128 + lane)] = r.c;
    st[blk_swz(192 + lane)] = r.d;
    o[0] = st[blk_swz(4 * lane)];
    o[1] = st[blk_swz(4 * lane + 1)];
    o[2] = st[blk_swz(4 * lane + 2)];
    o[3] = st[blk_swz(4 * lane + 3)];
}
