// msa_merge.hip -- multi-GPU count merge: export a counted table as key-hash
// partitions, import the partitions other GPUs sent (after an RCCL all-to-all).
//
// Replaces the reference's point-to-point merge (send_hash_table /
// receive_hash_table / ht_merge, parallel_spotify.c:152-158, 397-432, driven
// at 1011-1025), where every rank streams every key to rank 0 as three MPI
// messages and rank 0 re-inserts them serially.  Here each GPU owns the keys
// whose 64-bit hash falls in its partition, so the merge is one all-to-all
// and every GPU merges and ranks its own key range in parallel.
//
// Wire format, one block per destination partition:
//   header  32 B : u64 n_entries, u64 blob_bytes, u64 0, u64 0
//   records 32 B : u64 count, u32 len, u32 blob_off, u8 key[16] (first 16 bytes, 0-padded)
//   blob         : keys longer than 16 bytes, each padded to 16 B
// Keys are the final key bytes (words already lower-cased, artists as
// duplicate_field returned them).
#include "msa_internal.h"
#include "msa_tables.h"

namespace {
__device__ __forceinline__ u32 lower1m(u32 c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }
__device__ __forceinline__ u64 part_of(u64 h, u32 nparts) { return fmix64(h ^ 0xA5A5A5A55A5A5A5AULL) % nparts; }

// ctr[p] += v for every active lane, one atomic per distinct p in the wave
// (per-entry atomics on a handful of partition counters serialised at the
// L2: 400 us for 33K words into one partition).  Returns the lane's
// exclusive offset within its partition's claim.
__device__ __forceinline__ u64 wave_add(u64 *ctr, u32 p, u64 v) {
    const u32 lane = lane_id();
    u64 todo = __ballot(1);
    u64 mine = 0;
    while (todo) {
        const int lead = __ffsll((long long)todo) - 1;
        const u32 pl = __shfl(p, lead);
        const u64 grp = __ballot(p == pl) & todo;
        // this group's total and each member's exclusive prefix (v varies per lane)
        u64 pre = 0, tot = 0;
        for (u64 m = grp; m; m &= m - 1) {
            const int l = __ffsll((long long)m) - 1;
            const u64 vl = __shfl(v, l);
            if (l < (int)lane) pre += vl;
            tot += vl;
        }
        u64 base = 0;
        if ((int)lane == lead) base = atomicAdd((unsigned long long *)&ctr[pl], (unsigned long long)tot);
        base = __shfl(base, lead);
        if (p == pl && ((grp >> lane) & 1ull)) mine = base + pre;
        todo &= ~grp;
    }
    return mine;
}
}  // namespace

__device__ void exp_entry(const ExpSrc &x, u64 e, u64 *count, u32 *len, u64 *k0, u64 *k1, const u8 **lp,
                          int *lower) {
    *lp = nullptr;
    *lower = 0;
    *k0 = 0;
    *k1 = 0;
    if (x.d_K1) {  // dense entries first, then the long words (ns = nm = 0)
        if (e < x.nd) {
            *k0 = __builtin_bswap64(x.d_K1[e]);
            *k1 = __builtin_bswap64(x.d_K0[e]);
            *count = x.d_cnt[e];
            u32 n = 0;
            while (n < 16 && (((n < 8 ? *k0 : *k1) >> (8 * (n & 7))) & 0xFF)) ++n;
            *len = n;
            return;
        }
        e -= x.nd;
    }
    if (x.artists) {
        const u64 slot = x.a_list[e];
        *count = x.a_tab[4 * slot + 1];
        const u64 rep = x.a_tab[4 * slot + 2];
        *len = x.key_len[rep];
        *lp = x.arena + x.key_off[rep];
        return;
    }
    if (e < x.ns) {
        const u64 slot = x.s_list[e];
        const u64 w0 = x.s_tab[2 * slot];
        *k0 = w0 & TAB_KEY7;
        *count = x.s_tab[2 * slot + 1] + tab_gather8(w0);
        u32 n = 0;
        while (n < 8 && ((*k0 >> (8 * n)) & 0xFF)) ++n;
        *len = n;
    } else if (e < x.ns + x.nm) {
        const u64 slot = x.m_list[e - x.ns];
        const u64 w0 = x.m_tab[4 * slot];
        *k0 = w0 & TAB_KEY7;
        *k1 = x.m_tab[4 * slot + 1];
        *count = x.m_tab[4 * slot + 2] + tab_gather8(w0);
        u32 n = 8;
        while (n < 16 && ((*k1 >> (8 * (n - 8))) & 0xFF)) ++n;
        *len = n;
    } else {
        const u64 slot = x.l_list[e - x.ns - x.nm];
        *count = x.l_tab[4 * slot + 1] + 1;  // h_insert IMPL1
        const u64 rep = x.l_tab[4 * slot + 2];
        *len = x.l_len[rep];
        *lp = tok_at(x.buf, x.extra, x.l_pos[rep]);
        *lower = 1;
    }
}

__device__ __forceinline__ void key16_from(const u8 *lp, u32 len, int lower, u64 *k0, u64 *k1) {
    u64 a = 0, b = 0;
    for (u32 i = 0; i < 16 && i < len; ++i) {
        u64 ch = lower ? lower1m(lp[i]) : lp[i];
        if (i < 8) a |= ch << (8 * i);
        else b |= ch << (8 * (i - 8));
    }
    *k0 = a;
    *k1 = b;
}

__device__ u64 exp_hash(u64 k0, u64 k1, u32 len, const u8 *lp, int lower) {
    if (len <= 16) return fmix64(k0 ^ fmix64(k1 ^ len));
    return bytes_hash(lp, len, lower);
}

// pass A: per-partition entry counts and blob bytes
__global__ void k_exp_count(ExpSrc x, u64 n, u32 nparts, u64 *pcnt, u64 *pblob) {
    const u64 e = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    u64 count, k0, k1;
    u32 len;
    const u8 *lp;
    int lower;
    exp_entry(x, e, &count, &len, &k0, &k1, &lp, &lower);
    if (lp) key16_from(lp, len, lower, &k0, &k1);
    const u32 p = (u32)part_of(exp_hash(k0, k1, len, lp, lower), nparts);
    (void)wave_add(pcnt, p, 1);
    (void)wave_add(pblob, p, len > 16 ? (u64)((len + 15) & ~15u) : 0);
}

// pass B: write the records.  pbase[p] = byte offset of partition p's block;
// cursors (zeroed) hand out record slots and blob space within a block.
__global__ void k_exp_write(ExpSrc x, u64 n, u32 nparts, const u64 *pbase, const u64 *pcnt, u64 *rcur, u64 *bcur,
                            u8 *out) {
    const u64 e = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    u64 count, k0, k1;
    u32 len;
    const u8 *lp;
    int lower;
    exp_entry(x, e, &count, &len, &k0, &k1, &lp, &lower);
    if (lp) key16_from(lp, len, lower, &k0, &k1);
    const u32 p = (u32)part_of(exp_hash(k0, k1, len, lp, lower), nparts);
    const u64 i = wave_add(rcur, p, 1);
    u8 *blk = out + pbase[p];
    const u64 boff = wave_add(bcur, p, len > 16 ? (u64)((len + 15) & ~15u) : 0);
    if (len > 16) {
        u8 *dst = blk + 32 + 32 * pcnt[p] + boff;
        for (u32 k = 0; k < len; ++k) dst[k] = (u8)(lower ? lower1m(lp[k]) : lp[k]);
    }
    u64 *rec = reinterpret_cast<u64 *>(blk + 32 + 32 * i);
    rec[0] = count;
    rec[1] = (u64)len | (boff << 32);
    rec[2] = k0;
    rec[3] = k1;
}

__global__ void k_exp_headers(u32 nparts, const u64 *pbase, const u64 *pcnt, const u64 *pblob, u8 *out) {
    const u32 p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= nparts) return;
    u64 *h = reinterpret_cast<u64 *>(out + pbase[p]);
    h[0] = pcnt[p];
    h[1] = pblob[p];
    h[2] = 0;
    h[3] = 0;
}

// ---------------------------------------------------------------------------
// Import.  blk_off[0..nblk] = byte offsets of the received blocks (last = end);
// rec_base[b] = index of block b's first record among all received records.
__global__ void k_imp_index(const u8 *in, const u64 *blk_off, u32 nblk, u64 *rec_base) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    u64 acc = 0;
    for (u32 b = 0; b < nblk; ++b) {
        rec_base[b] = acc;
        if (blk_off[b + 1] > blk_off[b]) acc += reinterpret_cast<const u64 *>(in + blk_off[b])[0];
    }
    rec_base[nblk] = acc;
}

__global__ void k_imp_insert(const u8 *in, const u64 *blk_off, const u64 *rec_base, u32 nblk, ImpDst d) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rec_base[nblk]) return;
    u32 b = 0;
    while (b + 1 < nblk && rec_base[b + 1] <= r) ++b;
    const u8 *blk = in + blk_off[b];
    const u64 nrec_b = reinterpret_cast<const u64 *>(blk)[0];
    const u64 li = r - rec_base[b];
    const u64 *rec = reinterpret_cast<const u64 *>(blk + 32 + 32 * li);
    const u64 count = rec[0];
    const u32 len = (u32)(rec[1] & 0xFFFFFFFFu);
    const u64 boff = rec[1] >> 32;
    const u64 k0 = rec[2], k1 = rec[3];
    // key bytes: inline (record) or blob; positions are offsets into `in`
    const u64 kpos = (len > 16) ? (blk_off[b] + 32 + 32 * nrec_b + boff) : (blk_off[b] + 32 + 32 * li + 16);
    if (d.artists) {
        d.key_off[r] = kpos;
        d.key_len[r] = len;
        u64 h = bytes_hash(in + kpos, len, 0);
        d.key_slot[r] = h_insert(d.a_tab, d.a_mask, h, count, r, d.a_list, d.a_list_cap, &d.ctr->a_claimed, d.ctr,
                                 OVF_A);
        return;
    }
    if (len <= 8) {
        s_insert(d.s_tab, d.s_mask, k0, count, d.s_list, d.s_list_cap, d.ctr);
    } else if (len <= 16) {
        m_insert(d.m_tab, d.m_mask, k0, k1, count, d.m_list, d.m_list_cap, d.ctr);
    } else {
        const u64 i = atomicAdd((unsigned long long *)&d.ctr->l_occ, 1ull);
        if (i >= d.l_cap) {
            atomicOr((unsigned long long *)&d.ctr->overflow, (unsigned long long)OVF_L);
            return;
        }
        d.l_pos[i] = kpos | MSA_POS_EXTRA;
        d.l_len[i] = len;
        const u64 h = bytes_hash(in + kpos, len, 1);
        d.l_slot[i] = h_insert<true, true>(d.l_tab, d.l_mask, h, count, i, d.l_list, d.l_list_cap, &d.ctr->l_claimed, d.ctr,
                               OVF_LT);
    }
}

// ---------------------------------------------------------------------------
// Ranked export: entries [0, n) of a ranked table (rank order) as ONE block of
// the wire format above, so that a root GPU can import the blocks of every
// GPU (disjoint key partitions) and rank their union -- the global ranking, or
// its top-k when every GPU sent its own top-k.  The blob is the ranked key
// blob itself (keys unpadded; the importer reads long keys byte by byte).
__global__ void k_exp_ranked(const u64 *__restrict__ counts, const u64 *__restrict__ off, const u8 *__restrict__ blob,
                             u64 n, u64 blob_end, u8 *__restrict__ out) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) {
        u64 *h = reinterpret_cast<u64 *>(out);
        h[0] = n;
        h[1] = blob_end;
        h[2] = 0;
        h[3] = 0;
    }
    if (i >= n) return;
    const u64 o = off[i], e = (i + 1 < n) ? off[i + 1] : blob_end;
    const u32 len = (u32)(e - o);
    u64 k0 = 0, k1 = 0;
    if (len <= 16) {
        for (u32 k = 0; k < len; ++k) {
            const u64 ch = blob[o + k];
            if (k < 8) k0 |= ch << (8 * k);
            else k1 |= ch << (8 * (k - 8));
        }
    }
    u64 *rec = reinterpret_cast<u64 *>(out + 32 + 32 * i);
    rec[0] = counts[i];
    rec[1] = (u64)len | (o << 32);
    rec[2] = k0;
    rec[3] = k1;
}

// ---------------------------------------------------------------------------
static inline dim3 g1(u64 n, u32 t = 256) { return dim3((u32)((n + t - 1) / t)); }

hipError_t msa_launch_exp_count(const ExpSrc &x, u64 n, u32 nparts, u64 *pcnt, u64 *pblob, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_exp_count, g1(n), dim3(256), 0, s, x, n, nparts, pcnt, pblob);
    return hipGetLastError();
}
hipError_t msa_launch_exp_write(const ExpSrc &x, u64 n, u32 nparts, const u64 *pbase, const u64 *pcnt,
                                const u64 *pblob, u64 *rcur, u64 *bcur, u8 *out, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_exp_write, g1(n), dim3(256), 0, s, x, n, nparts, pbase, pcnt, rcur, bcur, out);
    hipLaunchKernelGGL(k_exp_headers, g1(nparts, 64), dim3(64), 0, s, nparts, pbase, pcnt, pblob, out);
    return hipGetLastError();
}
hipError_t msa_launch_imp(const u8 *in, const u64 *blk_off, u32 nblk, u64 *rec_base, u64 nrec_total, const ImpDst &d,
                          hipStream_t s) {
    hipLaunchKernelGGL(k_imp_index, dim3(1), dim3(64), 0, s, in, blk_off, nblk, rec_base);
    if (nrec_total) hipLaunchKernelGGL(k_imp_insert, g1(nrec_total), dim3(256), 0, s, in, blk_off, rec_base, nblk, d);
    return hipGetLastError();
}
hipError_t msa_launch_exp_ranked(const u64 *counts, const u64 *off, const u8 *blob, u64 n, u64 blob_end, u8 *out,
                                 hipStream_t s) {
    hipLaunchKernelGGL(k_exp_ranked, g1(n ? n : 1), dim3(256), 0, s, counts, off, blob, n, blob_end, out);
    if (blob_end) (void)hipMemcpyAsync(out + 32 + 32 * n, blob, blob_end, hipMemcpyDeviceToDevice, s);
    return hipGetLastError();
}
