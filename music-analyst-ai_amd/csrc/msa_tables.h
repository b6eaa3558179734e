// msa_tables.h -- open-addressing count tables in HBM (device code).
//
// Replaces the reference's HashTable/ht_put (parallel_spotify.c:47-149), which
// keys by strdup'ed strings.  Keys here are exact and fixed-width:
//   S-table  words of 1..8 bytes  : key = the 8 lower-cased bytes (LE, 0-pad)
//                                   slot = {key u64, count u64}   16 B
//   M-table  words of 9..16 bytes : key = two such words
//                                   slot = {k0, k1, count, 0}     32 B
//   H-table  anything longer (rare words, artist names): key = 64-bit hash,
//            slot = {hash, count, rep}; rep = index of the first occurrence,
//            every occurrence is later byte-compared against rep, so a hash
//            collision is detected, never silently merged.
// All shared words are touched with device-scope atomics only (no plain loads
// of another CU's writes: per-XCD L2s are not coherent).
#pragma once
#include "msa_internal.h"

// Linear probing: a table holds at most half as many keys as slots (its slot
// list's capacity), where the longest probe runs stay far below this; an
// insert that probes this far finds the table (nearly) full -- overflow, and
// the stage repeats with a larger table.  (4096 let a full table take
// thousands of L2 atomics per insert before the first one gave up.)
#define MSA_MAX_PROBE 512u

// A table that overflowed is full: every later insert into it would probe up
// to MSA_MAX_PROBE slots with an L2 atomic each (a cold run on a
// high-cardinality input spent seconds in such inserts before the retry that
// grows the table).  Every 16 probes an insert checks the table's overflow bit
// and gives up once it is set -- the stage is repeated with a larger table
// anyway; an insert that finds its slot within 16 probes never reads it.
__device__ __forceinline__ bool table_full(u32 probe, const Counters *ctr, u64 ovf_bit) {
    return (probe & 15u) == 15u &&
           (__hip_atomic_load(const_cast<u64 *>(&ctr->overflow), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ovf_bit) != 0;
}

// S / M keys are lower-cased token bytes (< 0x80) and zero padding, so bit 7
// of every byte of the first key word is free: a claim writes the key with a
// count of at most 255 spread over those bits (bit j of the count -> bit
// 8 j + 7), one CAS for a new key instead of a claim and a count add (the
// high-cardinality inserts are at the memory-side atomic rate).  A slot's
// count = its count word + the bits of its first key word; the key = that
// word & TAB_KEY7.
#define TAB_KEY7 0x7F7F7F7F7F7F7F7Full
__host__ __device__ __forceinline__ u64 tab_spread8(u64 c) {  // c < 256
    u64 r = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) r |= ((c >> j) & 1ull) << (8 * j + 7);
    return r;
}
__host__ __device__ __forceinline__ u64 tab_gather8(u64 w) {  // bit 8 j + 7 -> bit j
    u64 r = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) r |= ((w >> (8 * j + 7)) & 1ull) << j;
    return r;
}
// the claim value of a key word and the count left for the count word
#ifndef TAB_EMBED
#define TAB_EMBED 1  // 0: the key alone, the count always by an add (A/B builds)
#endif
__device__ __forceinline__ u64 tab_claim(u64 k0, u64 cnt, u64 *rest) {
    if (TAB_EMBED && cnt < 256) {
        *rest = 0;
        return k0 | tab_spread8(cnt);
    }
    *rest = cnt;
    return k0;
}

// Probe by CAS straight away (the CAS returns the slot's key: one L2 atomic
// per probe) instead of an atomic load first and a CAS only on an empty slot
// (two for every new key: the high-cardinality inserts).  TAB_CAS_FIRST=0
// builds the load-first probe.  A key inserted once per occurrence (an
// aggregation table that is full) probes load-first: on a hot key a CAS
// that fails is still a serialised read-modify-write at the L2.
#ifndef TAB_CAS_FIRST
#define TAB_CAS_FIRST 1
#endif
template <bool CASF = (TAB_CAS_FIRST != 0)>
__device__ __forceinline__ u64 probe_word(u64 *p, u64 key) {
    if (CASF) return atomicCAS((unsigned long long *)p, 0ull, (unsigned long long)key);
    const u64 cur = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return cur ? cur : atomicCAS((unsigned long long *)p, 0ull, (unsigned long long)key);
}

__device__ __forceinline__ u64 ld_relaxed(const u64 *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Append the slots the calling lanes claimed to a table's dense slot list:
// one claim-counter atomic per wave, not per key (a same-address atomic per
// new key serialised at the L2: 5 M new long words took 3.8 ms).  Called by
// every lane that ran the insert, after its probe loop (reconverged).
__device__ __forceinline__ void list_append_wave(bool isnew, u64 slot, u32 *list, u64 list_cap, u64 *claimed,
                                                 Counters *ctr, u64 ovf_bit) {
    const u64 B = __ballot(isnew);
    if (!B) return;
    const int leader = __ffsll((long long)B) - 1;
    u64 base = 0;
    if ((int)lane_id() == leader) base = atomicAdd((unsigned long long *)claimed, (unsigned long long)__popcll(B));
    base = readlane64(base, leader);
    if (isnew) {
        const u64 i = base + mbcnt(B);
        if (i < list_cap) list[i] = (u32)slot;
        else atomicOr((unsigned long long *)&ctr->overflow, (unsigned long long)ovf_bit);
    }
}

// Workgroup-staged list appends: new slots collect in LDS (one LDS add per
// wave), then stage_flush claims the list range with ONE device add per
// workgroup.  A full staging area falls back to a device claim per lane.
__device__ __forceinline__ void stage_new(bool isnew, u64 slot, u32 *staged, u32 *nst, u32 cap, u32 *list,
                                          u64 list_cap, u64 *claimed, Counters *ctr, u64 ovf_bit) {
    const u64 B = __ballot(isnew);
    if (!B) return;
    const int leader = __ffsll((long long)B) - 1;
    u32 base = 0;
    if ((int)lane_id() == leader) base = atomicAdd(nst, (u32)__popcll(B));
    base = __shfl(base, leader);
    if (!isnew) return;
    const u32 at = base + mbcnt(B);
    if (at < cap) {
        staged[at] = (u32)slot;
        return;
    }
    const u64 i = atomicAdd((unsigned long long *)claimed, 1ull);
    if (i < list_cap) list[i] = (u32)slot;
    else atomicOr((unsigned long long *)&ctr->overflow, (unsigned long long)ovf_bit);
}
// after a workgroup barrier that follows every stage_new of the workgroup
__device__ __forceinline__ void stage_flush(const u32 *staged, const u32 *nst, u32 cap, u64 *gbase, u32 *list,
                                            u64 list_cap, u64 *claimed, Counters *ctr, u64 ovf_bit) {
    const u32 m = min(*nst, cap);
    if (threadIdx.x == 0) *gbase = m ? atomicAdd((unsigned long long *)claimed, (unsigned long long)m) : 0ull;
    __syncthreads();
    for (u32 k = threadIdx.x; k < m; k += blockDim.x) {
        const u64 at = *gbase + k;
        if (at < list_cap) list[at] = staged[k];
        else atomicOr((unsigned long long *)&ctr->overflow, (unsigned long long)ovf_bit);
    }
}

// S-table insert; claimed slots are appended to `list` (dense, for ranking)
// unless LIST is false (the main scan: its lists are built afterwards by
// k_list_build, so new keys do not serialise on one claim counter).
template <bool LIST = true, bool CASF = (TAB_CAS_FIRST != 0)>
__device__ __forceinline__ void s_insert(u64 *tab, u64 mask, u64 key, u64 cnt, u32 *list,
                                         u64 list_cap, Counters *ctr) {
    u64 h = fmix64(key) & mask, rest;
    const u64 claim = tab_claim(key, cnt, &rest);
    bool isnew = false, found = false;
    for (u32 probe = 0; probe < MSA_MAX_PROBE; ++probe) {
        u64 *slot = tab + 2 * h;
        const u64 cur = probe_word<CASF>(slot, claim);
        if (cur == 0) {  // claimed with the count (or the count word takes it)
            if (rest) atomicAdd((unsigned long long *)(slot + 1), (unsigned long long)rest);
            isnew = found = true;
            break;
        }
        if ((cur & TAB_KEY7) == key) {
            atomicAdd((unsigned long long *)(slot + 1), (unsigned long long)cnt);
            found = true;
            break;
        }
        if (table_full(probe, ctr, OVF_S)) break;
        h = (h + 1) & mask;
    }
    if (!found) atomicOr((unsigned long long *)&ctr->overflow, (unsigned long long)OVF_S);
    if (LIST) list_append_wave(isnew, h, list, list_cap, &ctr->s_claimed, ctr, OVF_S);
}

// M-table insert (two-word key).  The slot is claimed by CAS on k0 and the
// winner then publishes k1; a prober that finds k0 equal but k1 still 0 simply
// retries that slot on its next loop trip (no spin inside a divergent branch,
// so a same-wave winner always gets to publish).  LIST as for s_insert.
template <bool LIST = true, bool CASF = (TAB_CAS_FIRST != 0)>
__device__ __forceinline__ void m_insert(u64 *tab, u64 mask, u64 k0, u64 k1, u64 cnt, u32 *list,
                                         u64 list_cap, Counters *ctr) {
    u64 h = fmix64(k0 ^ fmix64(k1)) & mask, rest;
    const u64 claim = tab_claim(k0, cnt, &rest);
    u32 probe = 0, spins = 0;
    bool isnew = false, found = false;
    while (probe < MSA_MAX_PROBE) {
        u64 *slot = tab + 4 * h;
        const u64 c0 = probe_word<CASF>(slot, claim);
        if (c0 == 0) {
            __hip_atomic_store(slot + 1, k1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (rest) atomicAdd((unsigned long long *)(slot + 2), (unsigned long long)rest);
            isnew = found = true;
            break;
        }
        if ((c0 & TAB_KEY7) == k0) {
            u64 c1 = ld_relaxed(slot + 1);
            if (c1 == 0) {  // claimed, k1 not yet visible: retry this slot
                if (++spins > (1u << 24)) break;
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            if (c1 == k1) {
                atomicAdd((unsigned long long *)(slot + 2), (unsigned long long)cnt);
                found = true;
                break;
            }
        }
        if (table_full(probe, ctr, OVF_M)) break;
        h = (h + 1) & mask;
        ++probe;
    }
    if (!found) atomicOr((unsigned long long *)&ctr->overflow, (unsigned long long)OVF_M);
    if (LIST) list_append_wave(isnew, h, list, list_cap, &ctr->m_claimed, ctr, OVF_M);
}

// H-table insert by 64-bit hash; returns the slot index (or ~0 on overflow).
// The CAS winner records `rep`; readers only look at rep in a later kernel.
// LIST false: no list append; *isnew_out tells the caller (k_long_insert
// stages its new slots per workgroup: a claim per wave on the one counter
// had serialised at the memory side)
// IMPL1 (the long-word table): a claimed slot counts one occurrence without
// an add -- its count word holds the occurrences past the first (readers add
// 1), so a new word's insert is a claim and the rep store, no count add
template <bool LIST = true, bool IMPL1 = false>
__device__ __forceinline__ u64 h_insert(u64 *tab, u64 mask, u64 hash, u64 cnt, u64 rep, u32 *list,
                                        u64 list_cap, u64 *claimed, Counters *ctr, u64 ovf_bit,
                                        bool *isnew_out = nullptr) {
    if (hash == 0) hash = 0x8000000000000000ULL;
    u64 h = hash & mask, res = ~0ull;
    bool isnew = false;
    for (u32 probe = 0; probe < MSA_MAX_PROBE; ++probe) {
        u64 *slot = tab + 4 * h;
        const u64 cur = probe_word(slot, hash);
        if (cur == 0) {
            __hip_atomic_store(slot + 2, rep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const u64 add = IMPL1 ? cnt - 1 : cnt;
            if (add) atomicAdd((unsigned long long *)(slot + 1), (unsigned long long)add);
            isnew = true;
            res = h;
            break;
        }
        if (cur == hash) {
            atomicAdd((unsigned long long *)(slot + 1), (unsigned long long)cnt);
            res = h;
            break;
        }
        if (table_full(probe, ctr, ovf_bit)) break;
        h = (h + 1) & mask;
    }
    if (res == ~0ull) atomicOr((unsigned long long *)&ctr->overflow, (unsigned long long)ovf_bit);
    if (LIST) list_append_wave(isnew, res, list, list_cap, claimed, ctr, ovf_bit);
    else *isnew_out = isnew;
    return res;
}

// Artist-key hashes of the lines shortcut (k_rec_spans -> k_artist_count):
// two independent 64-bit hashes, each a sum of per-position products of the
// key's little-endian 8-byte words (zero padded) folded by fmix64 every 32
// bytes -- cheap enough for one hash pair per record.  The word and byte
// forms agree for every key.
__host__ __device__ __forceinline__ u64 akey_fold(u64 h, u64 w0, u64 w1, u64 w2, u64 w3, int second) {
    if (!second)
        return fmix64(h + w0 * 0x9E3779B97F4A7C15ULL + w1 * 0xC2B2AE3D27D4EB4FULL + w2 * 0x165667B19E3779F9ULL +
                      w3 * 0xD6E8FEB86659FD93ULL);
    return fmix64(h ^ (w0 * 0xFF51AFD7ED558CCDULL + w1 * 0xC4CEB9FE1A85EC53ULL + w2 * 0x9FB21C651E98DF25ULL +
                       w3 * 0xBF58476D1CE4E5B9ULL));
}
__host__ __device__ __forceinline__ u64 akey_seed(u64 n, int second) {
    return second ? (0x6A09E667F3BCC909ULL ^ (n * 0xBB67AE8584CAA73BULL)) : (n * 0x94D049BB133111EBULL + 0x243F6A8885A308D3ULL);
}
__device__ __forceinline__ u64 akey_hash_bytes(const u8 *p, u64 n, int second) {
    u64 h = akey_seed(n, second);
    for (u64 b = 0; b < n || b == 0; b += 32) {
        u64 w[4] = {0, 0, 0, 0};
        for (u32 i = 0; i < 32 && b + i < n; ++i) w[i >> 3] |= (u64)p[b + i] << (8 * (i & 7));
        h = akey_fold(h, w[0], w[1], w[2], w[3], second);
        if (n == 0) break;
    }
    return h;
}

// H-table insert for artist keys with the second hash: sum2 (the sum of h2
// over the occurrences added) accumulates in the slot's 4th word, so the
// table can check sum2 == count * h2(rep) afterwards (k_artist_h2_check).
template <bool LIST = true>
__device__ __forceinline__ u64 h_insert2(u64 *tab, u64 mask, u64 hash, u64 cnt, u64 rep, u64 sum2, u32 *list,
                                         u64 list_cap, u64 *claimed, Counters *ctr, u64 ovf_bit, bool *isnew_out = nullptr) {
    if (hash == 0) hash = 0x8000000000000000ULL;
    u64 h = hash & mask, res = ~0ull;
    bool isnew = false;
    for (u32 probe = 0; probe < MSA_MAX_PROBE; ++probe) {
        u64 *slot = tab + 4 * h;
        const u64 cur = probe_word(slot, hash);
        if (cur == 0) {
            __hip_atomic_store(slot + 2, rep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            atomicAdd((unsigned long long *)(slot + 1), (unsigned long long)cnt);
            atomicAdd((unsigned long long *)(slot + 3), (unsigned long long)sum2);
            isnew = true;
            res = h;
            break;
        }
        if (cur == hash) {
            atomicAdd((unsigned long long *)(slot + 1), (unsigned long long)cnt);
            atomicAdd((unsigned long long *)(slot + 3), (unsigned long long)sum2);
            res = h;
            break;
        }
        if (table_full(probe, ctr, ovf_bit)) break;
        h = (h + 1) & mask;
    }
    if (res == ~0ull) atomicOr((unsigned long long *)&ctr->overflow, (unsigned long long)ovf_bit);
    if (LIST) list_append_wave(isnew, res, list, list_cap, claimed, ctr, ovf_bit);
    else *isnew_out = isnew;
    return res;
}

// 64-bit hash of a byte string (lower-cased when `lower`), for the H-table.
__device__ __forceinline__ u64 bytes_hash(const u8 *p, u64 n, int lower) {
    u64 h = 0x243F6A8885A308D3ULL ^ (n * 0x9E3779B97F4A7C15ULL);
    u64 acc = 0;
    u32 k = 0;
    for (u64 i = 0; i < n; ++i) {
        u32 c = p[i];
        if (lower && c >= 'A' && c <= 'Z') c += 32;
        acc |= (u64)c << (8 * k);
        if (++k == 8) {
            h = fmix64(h ^ acc) * 0x9E3779B97F4A7C15ULL;
            acc = 0;
            k = 0;
        }
    }
    h = fmix64(h ^ acc ^ ((u64)k << 59));
    return h;
}
