// msa_api.hip -- C ABI of libmsa_hip (include/msa_hip.h): buffer management and
// the stage order of one GPU's pipeline.  All data-path work is in kernels
// (msa_scan.hip, msa_post.hip); the host only sizes buffers from a handful of
// device counters and parses the single header record (the reference does the
// same serially on rank 0 before its timed region, parallel_spotify.c:788-819).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <errno.h>
#include <stdarg.h>
#include <algorithm>

#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "msa_hip.h"
#include "msa_internal.h"

// ---- launchers (msa_scan.hip / msa_post.hip)
hipError_t msa_launch_summary(const u8 *, u64, u64, u32, ChunkSum *, hipStream_t);
u32 msa_fn_blocks(u32 nchunks);
hipError_t msa_launch_fn(const ChunkSum *, u64, u32, Fn *, State *, Fn *, State, State *, State *, hipStream_t);
hipError_t msa_launch_scan(const ScanArgs &, int, hipStream_t);
hipError_t msa_launch_scan_csv(const ScanArgs &, hipStream_t);
hipError_t msa_launch_scan_tokens(const ScanArgs &, hipStream_t);
hipError_t msa_launch_miss_agg(const ScanArgs &, hipStream_t);
u64 msa_mb_hist_words(const ScanArgs &, u32);
u32 msa_scan_blocks(const ScanArgs &);
u32 msa_tok_wgcu();
hipError_t msa_launch_scan_fold(const ScanArgs &, u64 *, hipStream_t);
u32 msa_fold_tiles(u32);
hipError_t msa_launch_miss_buckets(const ScanArgs &, u64 *, u64 *, u64 *, u64 *, ulonglong2 *, hipStream_t);
hipError_t msa_exclusive_scan(const u64 *, u64, u64 *, u64 *, u64 *, hipStream_t);
hipError_t msa_launch_csv_lines(int, const u64 *, const u8 *, const u64 *, u64, u64, u64, int, u64 *, u64 *, u64 *,
                                u64 *, u8 *, hipStream_t);
hipError_t msa_exclusive_scan2(const u64 *, u64, u64 *, u64 *, u64 *, const u64 *, u64, u64 *, u64 *, u64 *,
                               hipStream_t);
hipError_t msa_launch_rec_spans(const u8 *, const u64 *, const u32 *, u64, u64, int, u64 *, u64 *, u32 *, u64 *, u64 *,
                                u32 *, Counters *, const AKeys &, const u64 *, const u64 *, const u64 *, u64 *, int,
                                hipStream_t, hipEvent_t);
hipError_t msa_launch_artist_count(const u64 *, const u32 *, const u64 *, const u64 *, u64, u64 *, u64, u32 *, u64,
                                   Counters *, int, int, ulonglong2 *, u32 *, u32, hipStream_t);
hipError_t msa_launch_first_end(const u8 *, u64, u32, u32, u64 *, hipStream_t);
hipError_t msa_launch_quote_parity(const u8 *, u64, u32 *, hipStream_t);
hipError_t msa_launch_artist_verify(const u8 *, const u64 *, const u32 *, const u64 *, u64, const u64 *, Counters *,
                                    hipStream_t);
hipError_t msa_launch_long_verify(const u8 *, const u8 *, const u64 *, const u32 *, const u64 *, u64, const u64 *,
                                  Counters *, hipStream_t);
hipError_t msa_launch_exp_count(const ExpSrc &, u64, u32, u64 *, u64 *, hipStream_t);
hipError_t msa_launch_exp_write(const ExpSrc &, u64, u32, const u64 *, const u64 *, const u64 *, u64 *, u64 *, u8 *,
                                hipStream_t);
hipError_t msa_launch_exp_ranked(const u64 *, const u64 *, const u8 *, u64, u64, u8 *, hipStream_t);
hipError_t msa_launch_imp(const u8 *, const u64 *, u32, u64 *, u64, const ImpDst &, hipStream_t);
hipError_t msa_launch_col_write(int, const u8 *, const u64 *, const u64 *, const u64 *, const u32 *, u64, u64,
                                const u64 *, u8 *, const u8 *, const u64 *, const u32 *, hipStream_t);
hipError_t msa_launch_artist_key(const u8 *, const u64 *, const u64 *, const u64 *, u64, u64, u8 *, u64 *, u32 *, u64 *,
                                 u64 *, u64, u32 *, u64, Counters *, u64, int, int, hipStream_t);
hipError_t msa_launch_long(const u8 *, u64, const u8 *, u64, const u64 *, u64, u32 *, u64 *, u64 *, u64, u32 *, u64,
                           Counters *, hipStream_t);
hipError_t msa_launch_word_entries(const EntryArgs &, hipStream_t);
u64 msa_dn_vary_words();
hipError_t msa_launch_list_build(const u64 *, u64, u32, u32 *, u64, u64 *, Counters *, u64, hipStream_t);
hipError_t msa_launch_artist_entries(const u64 *, const u32 *, u64, const u8 *, const u64 *, const u32 *, u64 *, u64 *,
                                     u64 *, u32 *, u64 *, u64 *, hipStream_t);
u64 msa_radix_scratch_bytes(u64 n);
hipError_t msa_radix_sort(u64 *const[3], u64 *const[3], u64 *const[3], u32 *const[3], u64, int *, u8 *, hipStream_t,
                          const u64 * = nullptr, bool = true, const u64 * = nullptr, u32 = 0, u64 ** = nullptr,
                          u32 ** = nullptr);
u64 msa_comp_scratch_bytes();
hipError_t msa_radix_sort_comp(u64 *const[3], u64 *const[3], u64 *const[3], u32 *const[3], u64, int *, u8 *,
                               hipStream_t, const u64 *, u64 *, u8 *, u32 *, u64 **, u32 **);
hipError_t msa_comp_finish(u64 *, u64, const u8 *, u32, hipStream_t);
u64 msa_tie_blocks(u64);
hipError_t msa_launch_tie_count(const u64 *, const u64 *, const u64 *, u64, u64 *, u64 *, u64 *, hipStream_t);
hipError_t msa_launch_tie_seg(const u64 *, const u64 *, const u64 *, const u32 *, u64, u64 *, u64 *, u64 *, u32 *,
                              hipStream_t);
hipError_t msa_launch_tie_build(const u64 *, const u64 *, const u64 *, u64, const u64 *, const u64 *, const u32 *,
                                const u64 *, u32, const u64 *, const u64 *, const u64 *, const u8 *, const u8 *,
                                const u64 *, const u32 *, const u8 *, const u64 *, const u32 *, u64 *, u64 *, u64 *,
                                u32 *, u32 *, u64 *, hipStream_t);
hipError_t msa_launch_tie_apply(const u32 *, const u32 *, const u64 *, u64, u32 *, u32 *, u64 *, const u64 *,
                                const u64 *, u64 *, u64 *, hipStream_t);
hipError_t msa_launch_sort(u64 *const[3], u64 *const[3], u64 *const[3], u32 *const[3], u64, int *, hipStream_t);
hipError_t msa_launch_fixup(const u64 *, const u64 *, const u64 *, const u32 *, u64, const u64 *, const u8 *,
                            const u8 *, const u64 *, const u32 *, const u8 *, const u64 *, const u32 *, u32 *, hipStream_t);
u64 msa_rank_small_max();
hipError_t msa_launch_merge_ranked(const u8 *, const u64 *, const u64 *, u32, u64, const u64 *, u32, u64 *, u64 *,
                                   u64 *, u64 *, u64 *, u32 *, u64 *, u64 *, u64 *, u64 *, hipStream_t);
hipError_t msa_launch_merge_blob(const u32 *, u64, const u8 *, const u64 *, const u64 *, const u64 *, u8 *, u64 *,
                                 hipStream_t);
u64 msa_rank_small_scratch(u64 n);
hipError_t msa_launch_rank_small(u64 *const[3], u64 *const[3], u64 *const[3], u32 *const[3], u64, const u64 *,
                                 const u8 *, const u8 *, const u64 *, const u32 *, const u8 *, const u64 *,
                                 const u32 *, u32 *, u64 *, u64 *, u64 *, u64 *, u32 *, hipStream_t);
hipError_t msa_launch_blob(const u32 *, u64, const u64 *, const u64 *, const u64 *, const u64 *, const u8 *,
                           const u8 *, const u64 *, const u32 *, const u8 *, const u64 *, const u32 *, u64 *, u64 *, u64 *, u64 *,
                           u8 *, u64 *, u64, hipStream_t, int, const u64 *, const u64 *, const u64 *, u64);

#ifndef MSA_LISTS_BEFORE_SPANS
#define MSA_LISTS_BEFORE_SPANS 1  // 0: the library stream waits for the spans before the word lists (A/B builds)
#endif
#ifndef MSA_ARTIST_EARLY
#define MSA_ARTIST_EARLY 1  // 0: the split's artist pass waits for the offset scans too (A/B builds)
#endif
#ifndef MSA_ARTIST_SIDE
#define MSA_ARTIST_SIDE 1  // 0: the split's artist pass on the library stream, text.csv forked after it (A/B builds)
#endif
#ifndef MSA_ARTIST_SIDE_DENSE
#define MSA_ARTIST_SIDE_DENSE 0  // 1: MSA_ARTIST_SIDE for dense splits too (A/B builds)
#endif

// ---------------------------------------------------------------------------
namespace {

// Room before a text column's body for its header line (a label of at most
// 127 bytes + '\n', msa_summary's text_label): the body can be written
// before the header is known.
static const u64 kColHdrRoom = 256;

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    template <class T> T *as() const { return reinterpret_cast<T *>(p); }
};

struct BlobArgs {  // key sources of the last blob pass (for a rewrite after growth)
    const u8 *wbuf, *wextra, *arena;
    const u64 *key_off;
    const u32 *key_len;
    const u64 *ks2, *ks1, *ks0;  // the sorted key planes (null: read the keys through order)
    u64 lthr;                    // entries below: S/M words (the key is K1/K0)
};
struct RefineBufs {
    DevBuf sort_scratch;
    DevBuf t_head, t_tie, t_runid, t_tpos, t_bsum, t_total, t_K[3][3], t_V[3], t_Vn, t_Pn, t_Vc, t_Pc;
};

struct Ranked {
    DevBuf K[3][3];  // [set][k2,k1,k0]: set 0 = input, 1/2 = ping-pong
    DevBuf V[3];
    DevBuf ref, cnt, order, len, off, blob, counts;
    DevBuf scan_bsum, scan_total;  // the blob offsets' scan scratch (the two tables rank concurrently)
    DevBuf rank_cnt;               // the small-table ranking's per-tile counts
    u64 n = 0, blob_len = 0, blob_cap = 0;
    u64 lthr = 0;  // words: entries [0, lthr) are S/M keys (k_word_entries' order)
    DevBuf vary;   // the key planes' OR / AND over the entries (k_word_entries), for the radix sort
    DevBuf comp, cset;  // words: the composite sort keys and the distinct-count set (msa_radix_sort_comp)
    bool vary_ok = false;
    bool blob_pending = false;  // blob_len not read back yet (do_rank's sync)
    BlobArgs pending{};
    std::vector<u64> h_counts, h_off;
    std::vector<char> h_blob;
    bool host_valid = false;
};

u64 next_pow2(u64 v) {
    u64 p = 1;
    while (p < v) p <<= 1;
    return p;
}

// Pipeline stages timed with HIP events when profiling is on.
enum {
    ST_CSV_SUMMARY = 0,  // K1 + K2 over the CSV (chunk functions + prefix)
    ST_CSV_SCAN,         // K3: records, fields, lyric tokens -> word tables
    ST_ARTIST_COLUMN,    // artist.csv materialisation
    ST_TEXT_COLUMN,      // text.csv materialisation
    ST_ARTIST_SUMMARY,   // K1 + K2 over artist.csv
    ST_ARTIST_SCAN,      // K3 (records only) over artist.csv
    ST_ARTIST_KEYS,      // duplicate_field + artist table
    ST_LONG_WORDS,       // > 16-byte words: hash table + verification
    ST_RANK_WORDS,       // entries + sort + key blob, words
    ST_RANK_ARTISTS,     // the same, artists
    ST_MISS_AGG,         // K3's logged LDS-table misses -> word tables (k_miss_agg)
    ST_REC_SPANS,        // both columns' line spans + artist keys (k_rec_fast / k_rec_fix) + offset scans
    ST_CSV_TOKENS,       // split scan, second kernel: lyric tokens -> word tables (k_scan_tokens)
    ST_REC_FAST,         // k_rec_fast alone (inside ST_REC_SPANS)
    ST_COUNT_
};
const char *const kStageName[ST_COUNT_] = {"csv_summary", "csv_scan",    "artist_column", "text_column",
                                           "artist_summary", "artist_scan", "artist_keys",  "long_words",
                                           "rank_words",  "rank_artists", "csv_miss_agg", "rec_spans",
                                           "csv_tokens",  "rec_fast"};

struct ProfStage {
    hipEvent_t a = nullptr, b = nullptr;
    bool pending = false;
    double ms = 0;
    u64 launches = 0, bytes = 0, pend_bytes = 0;
};

}  // namespace

struct msa_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    std::mutex err_mu;
    // input
    DevBuf in_own;
    const u8 *in = nullptr;  // the segment processed (a view of the input)
    u64 n = 0;
    const u8 *in_base = nullptr;  // the loaded / bound input itself
    u64 n_base = 0;
    bool cont = false;  // continuation shard: no header row (multi-GPU)
    u64 a_beg = 0, a_end = 0;  // artist.csv segment the artist pass reads
    // multi-GPU merge
    DevBuf exp_buf, exp_meta, imp_w, imp_a, imp_meta;
    u64 exp_bytes = 0;
    bool merged_w = false, merged_a = false;
    // tables (bit 0 words, bit 1 artists) whose ranking is msa_import_ranked's
    // merge of received blocks: the count tables still hold this GPU's own
    // keys, so the table is ranked-only until the next split / partition import
    int ranked_only = 0;
    u64 split_attempts = 0;  // diagnostic (msa_debug_stat "split_attempts")
    // scan scratch
    DevBuf sums, carry, btot, bstate, small;  // small: Fn total + 2 States + ...
    // CSV records
    DevBuf rec_start, nulrel;  // rec_start[nrec] = end of the last record
    DevBuf alog, alog_n;            // artist count flush logs (k_artist_merge)
    DevBuf f0, tss, tse, span_fix;  // K3's per-record span events (k_rec_fast), listed exact-path records
    bool spans = false;             // the last scan recorded f0 / tss / tse
    u64 nrec = 0, rec_cap = 0;
    bool have_text_arrays = false;
    // side buffer: text.csv header-label remainder read back as lyrics
    DevBuf extra;
    u64 extra_len = 0;
    // columns
    DevBuf acol, alen, aoff, asrc, apairs, tcol, tlen, toff, tsrc, tpairs, scan_bsum, scan_total, tscan_bsum;
    int cus = 256;
#ifdef MSA_DIAG
    int ablate = 0;  // env MSA_ABLATE (diagnostic builds only, make variant): kernel ablations, results invalid
#else
    static constexpr int ablate = 0;  // the product library has no ablation switch
#endif
    int sort_mode = 0;  // MSA_SORT: 0 by size, 1 merge sort, 2 radix sort
    // radix sort + tie refinement scratch, one set per concurrently ranked
    // table (rb[1]: the artists on their own host thread and stream)
    RefineBufs rb[2];
    DevBuf blob_tot;  // the two tables' key-blob lengths (device), read back once per msa_rank
    // tie refinement of the radix path: per-level marks/scans, the subset's
    // three key sets + values, and its order positions

    u64 acol_len = 0, a_hdr_getline = 0, a_hdr_len = 0, tcol_len = 0;
    u64 col_hdr[2] = {0, 0};        // header-line bytes of artist.csv / text.csv
    bool col_lens_pending = false;  // acol_len, tcol_len, a_end not read back yet
    // artist pass: true = the exact record reader over artist.csv (forced by
    // msa_set_artist_reader / an artist piece set for a shard); otherwise the
    // lines are the records unless the split found an unquoted artist field
    // holding a '"' (Counters::a_quoted) or the label holds a '\n'
    bool artist_exact = false;       // msa_set_artist_reader
    bool artist_piece_set = false;   // msa_segment_set(MSA_PIECE_ARTISTS) since the split
    bool artist_spec = false;        // the split ran the artist pass's first count (msa_count uses it)
    bool a_dirty = false;            // the artist table holds slots no list names (wiped before the next split)
    bool have_tcol = false;
    // artist.csv records + keys
    DevBuf ar_start, arena, key_off, key_len, key_slot, kh1, kh2;
    u64 a_long_cap = 0;  // long-key area of the lines shortcut (grows when it overflowed)
    u64 nrec_a = 0;
    // tables
    DevBuf s_tab, s_list, m_tab, m_list, l_pos, l_len, l_slot, l_tab, l_list, a_tab, a_list;
    DevBuf mlog, mlog_n;  // K3's logged LDS-table misses (k_miss_agg)
    // the bucketed aggregation of the logs (msa_launch_miss_buckets): tile
    // histograms, their scan, the bucketed entries
    DevBuf mb_hist, mb_off, mb_bsum, mb_tot, mb_out;
    // env MSA_MISS_BUCKETS: 0 never (default), 1 always, 2 when the last split
    // logged > mb_min misses.  Measured and not taken: configs[4] 32.5 vs 28.6
    // ms/step (the bucket scatter 2.0 ms, the bucket aggregation 8.0: one claim
    // and one add per distinct key, far fewer in flight than k_miss_agg's
    // per-entry inserts); configs[2] 4.38 vs 2.90 (profiles/r04_t36_*)
    int mb_mode = 0;
    u64 mb_min = 24000000;
    u64 mb_prev = 0;     // the last split's logged misses
    // Dense entries (k_mb_agg<true>): a split whose previous run counted at
    // least dense_min distinct 3..16-byte words (high cardinality) buckets its
    // logs and writes the words' ranking entries directly -- no HBM word
    // table inserts, slot lists, table clears or k_word_entries over them.
    // A multi-GPU shard exports its dense entries' key partitions from the
    // planes (fill_exp_src); the rank that imports a partition counts it in
    // its tables.  env MSA_DENSE=0 turns it off, MSA_DENSE_MIN sets the
    // threshold.
    bool dense_on = true;
    u64 dense_min = 4000000;
    u64 prev_distinct = 0;  // the last split's distinct S + M words
    bool have_hist = false; // prev_distinct is a split's count (not the context's first split)
    bool dense_w = false;   // the current split's words are dense entries (Ranked rw's planes)
    bool dense_veto = false;  // a dense split overflowed (a bucket past its LDS table): tables until the input changes
    bool sharded = false;     // msa_set_shard was called: a multi-GPU shard (diagnostic)
    DevBuf lmask;         // the split scan's lyric token-byte mask (k_scan_struct -> k_scan_tokens)
    u64 s_slots = 0, m_slots = 0, l_occ_cap = 0, lt_slots = 0, a_slots = 0;
    u64 s_used_prev = 0, m_used_prev = 0, lt_used_prev = 0, a_used_prev = 0;
    // Table capacities (log2 slots / occurrence capacity).  They start small --
    // a table that fits the Infinity Cache is much faster than one sized for
    // the worst case -- and grow only when a run reports an overflow of that
    // table (msa_run retries); the grown size is kept for later runs.
    u32 s_log2 = 0, m_log2 = 0, lt_log2 = 0, a_log2 = 0;
    u64 l_occ_want = 0;
    u64 l_occ_last = 0;  // the last split's long-word position reservations (sizes the waves' ranges)
    u64 mlog_want = 0;  // K3 log entries the last split needed (grown when a log partition filled)
    u64 mlog_test = 0;  // env MSA_MLOG_ENTRIES (tests): the logs' first size, so that they overflow
    u64 mlog_cap_last = 0;  // entries per partition of the last split's logs
    State fin_cache{};     // the last split's final reader state (MSA_ABLATE 16384)
    u64 fin_cache_n = 0;   // its input length + 1 (0: none)
    // counters
    DevBuf ctr;
    Counters h_ctr{};
    // results
    Ranked rw, ra;
    msa_summary sum{};
    int stage = 0;  // 0 none, 1 split, 2 counted, 3 ranked
    // text.csv is written on a side stream, overlapping the artist pass and
    // the ranking (nothing downstream of the split reads it); every entry
    // point that could touch its buffers joins it first (join_side)
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // the artist table is ranked on a stream of its own beside the word table
    // (both small-table sorts are launch/latency-bound chains)
    hipStream_t rank2 = nullptr;
    // artist.csv beside the ranking
    hipStream_t aux = nullptr;
    hipEvent_t ev_aux_fork = nullptr, ev_aux_join = nullptr;
    bool aux_pending = false;
    hipEvent_t ev_r2_fork = nullptr, ev_r2_join = nullptr;
    // split scan: k_scan_struct done (the spans may start) / the spans done
    hipEvent_t ev_scan_a = nullptr, ev_spans = nullptr;
    hipEvent_t ev_fix = nullptr;  // rank2: the artist keys written (k_rec_fast + k_rec_fix), before the offset scans
    hipEvent_t ev_art = nullptr;  // side stream: the split's artist pass done (MSA_ARTIST_SIDE)
    // the folded split scan (k_scan_fold): tile statuses (5 words a tile) behind
    // the ticket counter, the tickets taken so far, the status epoch
    // env MSA_FOLD=1 (opt-in: measured as fast as K1 + K2 + k_scan_struct, 0.85
    // vs 0.35 + 0.50 ms)
    int fold = 0;
    DevBuf fold_buf;
    u64 fold_tbase = 0;
    u32 fold_ep = 0;
    int comp_sort = 1;      // env MSA_COMP_SORT=0: the words' radix sort by K2 and K1 (no composite key)
    u64 csv_host_max = 1ull << 20;  // env MSA_CSV_HOST_MAX: msa_write_table_csv's host loop up to this many lines
    int tie_seg = 1;        // env MSA_TIE_SEG=0: every tie round through the radix sort (no k_tie_seg)
    // the K2 final-state read-back (launch_scan_fn / wait_scan_fn)
    hipEvent_t ev_fin = nullptr;
    State fin_init{};
    bool fin_pending = false;
    // text.csv is written on the side stream from the moment its record
    // spans exist (right after the split's scans): beside the split's
    // read-back, the artist pass and the ranking; every entry point that
    // could touch its buffers joins it first (join_side)
    bool side_pending = false;
    // the text column's body starts at kColHdrRoom, its header line right
    // before it (written once the header is read back): tcol + tcol_off
    u64 tcol_off = 0;
    // the body is launched after the artist pass of msa_count: on the side
    // stream beside the count read-back and the ranking, or on the library
    // stream by the first entry point that needs it.  Measured: launched right
    // after the split's span scans, the gather's full grid held every CU and
    // the read-back copies waited ~440 us for it; with a persistent grid of 2
    // workgroups per CU (room for the artist tables beside it) the gather
    // itself took 1.5-1.9 ms instead of 0.55
    bool text_deferred = false;
    // artist.csv waits until the artist pass of msa_count is enqueued (that
    // pass reads k_rec_fast's keys, not the column); entry points that read
    // acol launch it first
    bool artist_deferred = false;
    std::string artist_hdr;
    // pinned read-back area: the counters, states and header bytes a run reads
    // back are copied here asynchronously and waited for with one sync
    // (pageable destinations made every copy a round trip of its own)
    unsigned char *pin = nullptr;
    // word_counts.csv / top_artists.csv bytes (msa_write_table_csv): line
    // lengths, offsets and the scan's scratch, the lines, and two pinned
    // staging halves the host writes from while the next half is copied
    DevBuf csv_len, csv_pos, csv_bsum, csv_out;
    unsigned char *csv_pin = nullptr;
    // profiling
    bool prof = false;
    ProfStage ps[ST_COUNT_];
};

// Fold a finished stage's event pair into its accumulator (waits for it).
static void prof_harvest(msa_ctx *c, int id) {
    ProfStage &s = c->ps[id];
    if (!s.pending) return;
    float ms = 0;
    if (hipEventSynchronize(s.b) == hipSuccess && hipEventElapsedTime(&ms, s.a, s.b) == hipSuccess) {
        s.ms += ms;
        s.launches += 1;
        s.bytes += s.pend_bytes;
    }
    s.pending = false;
}
static void prof_begin(msa_ctx *c, int id, hipStream_t st = nullptr) {
    if (!c->prof) return;
    ProfStage &s = c->ps[id];
    prof_harvest(c, id);
    if (!s.a) {
        (void)hipEventCreate(&s.a);
        (void)hipEventCreate(&s.b);
    }
    (void)hipEventRecord(s.a, st ? st : c->stream);
}
// a stage whose end event the launcher records itself (between two kernels)
static hipEvent_t prof_end_event(msa_ctx *c, int id, u64 bytes) {
    if (!c->prof) return nullptr;
    ProfStage &s = c->ps[id];
    s.pend_bytes = bytes;
    s.pending = true;
    return s.b;
}
static void prof_end(msa_ctx *c, int id, u64 bytes, hipStream_t st = nullptr) {
    if (!c->prof) return;
    ProfStage &s = c->ps[id];
    (void)hipEventRecord(s.b, st ? st : c->stream);
    s.pend_bytes = bytes;
    s.pending = true;
}

// The side stream starts after everything enqueued on the main stream so far.
static hipError_t fork_side(msa_ctx *c) {
    hipError_t e = hipEventRecord(c->ev_fork, c->stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(c->side, c->ev_fork, 0);
    return e;
}
static int materialise_column(msa_ctx *c, bool text, u64 hdr, DevBuf &col, DevBuf &lenb, DevBuf &offb,
                              DevBuf &srcb, DevBuf &pairsb, hipStream_t st);
static int put_bytes(msa_ctx *c, u8 *dst, const std::string &b, hipStream_t st);
static int start_text_side(msa_ctx *c);
static int launch_text(msa_ctx *c, hipStream_t st);
// The deferred artist.csv pass on the library stream.
// beside: on the aux stream (forked from the library stream here), so that the
// ranking does not queue behind it; every later call (and join_side) orders
// the library stream after it again.
static hipError_t launch_artist_col(msa_ctx *c, bool beside = false) {
    if (!c->artist_deferred) {
        if (!beside && c->aux_pending) {
            c->aux_pending = false;
            return hipStreamWaitEvent(c->stream, c->ev_aux_join, 0);
        }
        return hipSuccess;
    }
    c->artist_deferred = false;
    hipStream_t st = c->stream;
    hipError_t e;
    if (beside) {
        if ((e = hipEventRecord(c->ev_aux_fork, c->stream)) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(c->aux, c->ev_aux_fork, 0)) != hipSuccess) return e;
        st = c->aux;
    }
    prof_begin(c, ST_ARTIST_COLUMN, st);
    if (put_bytes(c, c->acol.as<u8>(), c->artist_hdr, st) ||
        materialise_column(c, false, c->artist_hdr.size(), c->acol, c->alen, c->aoff, c->asrc, c->apairs, st))
        return hipErrorUnknown;
    prof_end(c, ST_ARTIST_COLUMN, c->nrec * 16 * 2, st);  // ~16-byte artist lines read + written
    if (beside) {
        if ((e = hipEventRecord(c->ev_aux_join, c->aux)) != hipSuccess) return e;
        c->aux_pending = true;
    }
    return hipGetLastError();
}
// Everything the library owes on its stream: a column pass not launched yet
// runs there, one on the side stream is waited for (enqueued, no host wait).
static hipError_t join_side(msa_ctx *c) {
    if (c->artist_deferred) {
        const hipError_t e = launch_artist_col(c);
        if (e != hipSuccess) return e;
    }
    if (c->text_deferred && launch_text(c, c->stream)) return hipErrorUnknown;
    if (c->aux_pending) {  // artist.csv beside the ranking
        c->aux_pending = false;
        const hipError_t e = hipStreamWaitEvent(c->stream, c->ev_aux_join, 0);
        if (e != hipSuccess) return e;
    }
    if (!c->side_pending) return hipSuccess;
    c->side_pending = false;
    return hipStreamWaitEvent(c->stream, c->ev_join, 0);
}

static int fail(msa_ctx *c, int code, const char *fmt, ...) {
    char b[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(b, sizeof b, fmt, ap);
    va_end(ap);
    if (c) {
        std::lock_guard<std::mutex> g(c->err_mu);  // the artists' ranking may fail on its own thread
        c->err = b;
    }
    return code;
}

#define HIPC(c, x)                                                                                      \
    do {                                                                                                \
        hipError_t e_ = (x);                                                                            \
        if (e_ != hipSuccess) return fail(c, MSA_ERR_HIP, "%s failed: %s (%s:%d)", #x, hipGetErrorString(e_), \
                                          __FILE__, __LINE__);                                          \
    } while (0)

// A buffer is freed only once no kernel can still touch it: work on the
// library's other streams (text.csv on the side stream, the spans / artist
// ranking on rank2) may be in flight when a host call grows a buffer, and
// memory hipFree returns can be handed out again at once.
static void free_quiet(void *p) {
    if (!p) return;
    (void)hipDeviceSynchronize();
    (void)hipFree(p);
}

static hipError_t ensure(DevBuf &b, size_t bytes, bool zero = false) {
    if (bytes == 0) bytes = 16;
    if (b.cap >= bytes) return hipSuccess;
    free_quiet(b.p);
    b.p = nullptr;
    b.cap = 0;
    size_t want = bytes + bytes / 4;
    hipError_t e = hipMalloc(&b.p, want);
    if (e != hipSuccess) return e;
    b.cap = want;
    // zeroed before any library stream can use it: the library's streams are
    // non-blocking, so nothing orders them after a null-stream memset -- wait
    // for it here
    if (zero && (e = hipMemset(b.p, 0, want)) == hipSuccess) e = hipDeviceSynchronize();
    return e;
}

static void release(DevBuf &b) {
    free_quiet(b.p);
    b.p = nullptr;
    b.cap = 0;
}

// ---------------------------------------------------------------- host CSV bits
// Header record parsing (parse_csv_line + duplicate_field with preserve = 0,
// parallel_spotify.c:258-304, 215-255) for the one header record.
static bool h_space(unsigned c) { return c == ' ' || (c >= 9 && c <= 13); }

static std::string h_dup_field(const unsigned char *f, size_t len) {
    size_t s = 0, e = len;
    while (s < len && h_space(f[s])) s++;
    while (e > s && h_space(f[e - 1])) e--;
    bool quoted = (e > s + 1 && f[s] == '"' && f[e - 1] == '"');
    size_t a = s, z = e;
    if (quoted) { a++; z--; }
    std::string r;
    for (size_t i = a; i < z; ++i) {
        if (f[i] == '"' && i + 1 < z && f[i + 1] == '"') { r.push_back('"'); i++; }
        else r.push_back((char)f[i]);
    }
    size_t x = 0, y = r.size();
    while (x < y && h_space((unsigned char)r[x])) x++;
    while (y > x && h_space((unsigned char)r[y - 1])) y--;
    return r.substr(x, y - x);
}

static bool h_parse_header(const unsigned char *rec, size_t len, std::string &a, std::string &t) {
    const void *z = memchr(rec, 0, len);
    if (z) len = (size_t)((const unsigned char *)z - rec);
    while (len > 0 && (rec[len - 1] == '\n' || rec[len - 1] == '\r')) len--;
    size_t comma[3];
    int nc = 0, q = 0;
    for (size_t i = 0; i < len && nc < 3; ++i) {
        if (rec[i] == '"') {
            if (q && i + 1 < len && rec[i + 1] == '"') i++;
            else q = !q;
        } else if (rec[i] == ',' && !q) {
            comma[nc++] = i;
        }
    }
    if (nc < 3) return false;
    a = h_dup_field(rec, comma[0]);
    t = h_dup_field(rec + comma[2] + 1, len - comma[2] - 1);
    return true;
}

// sanitize_header_name (parallel_spotify.c:510-543)
static void h_sanitize(const std::string &in, char *out) {
    size_t j = 0;
    for (unsigned char c : in) {
        if (c == '\n' || c == '\r') continue;
        if (j + 1 >= 128) continue;
        if (h_space(c)) out[j++] = '_';
        else if ((c >= '0' && c <= '9') || ((c | 0x20) >= 'a' && (c | 0x20) <= 'z') || c == '-' || c == '.' ||
                 c == '_')
            out[j++] = (char)c;
        else out[j++] = '_';
    }
    if (j == 0) { strcpy(out, "col"); return; }
    out[j] = 0;
}

// ------------------------------------------------------------------- scanning
// Scan a byte segment [b, e) of `buf`: K1 + K2 (+ K3 in `mode`).  Returns the
// reader state at the end of the segment in *fin.
// pin layout: [0, 512) Counters, [512, 1024) a state / small values, [1024, 1024 + kPinHead) header bytes
static const u64 kPinSmall = 512, kPinHead = 4096, kPinBytes = 1024 + kPinHead;
static_assert(sizeof(Counters) <= 512 && sizeof(State) <= 512, "pinned read-back layout");

// launch_scan_fn enqueues K1 + K2 and the read-back of the final state;
// wait_scan_fn waits for that read-back alone (work enqueued in between, such
// as a speculative K3, keeps running).
static int launch_scan_fn(msa_ctx *c, const u8 *buf, u64 b, u64 e, State init, int stage_id) {
    const u64 len = e > b ? e - b : 0;
    const u32 nch = (u32)((len + MSA_CHUNK - 1) / MSA_CHUNK);
    c->fin_init = init;
    c->fin_pending = nch != 0;
    if (!nch) return MSA_OK;
    HIPC(c, ensure(c->sums, sizeof(ChunkSum) * (size_t)(nch + 1)));
    HIPC(c, ensure(c->carry, sizeof(State) * (size_t)(nch + 1)));
    HIPC(c, ensure(c->btot, sizeof(Fn) * (size_t)(msa_fn_blocks(nch) + 1)));
    HIPC(c, ensure(c->bstate, sizeof(State) * (size_t)(msa_fn_blocks(nch) + 1)));
    HIPC(c, ensure(c->small, 4096));
    Fn *total = c->small.as<Fn>();
    State *d_fin = reinterpret_cast<State *>(c->small.as<char>() + 1024);
    prof_begin(c, stage_id);
    HIPC(c, msa_launch_summary(buf, b, e, nch, c->sums.as<ChunkSum>(), c->stream));
    HIPC(c, msa_launch_fn(c->sums.as<ChunkSum>(), b, nch, c->btot.as<Fn>(), c->bstate.as<State>(), total, init,
                          c->carry.as<State>(), d_fin, c->stream));
    prof_end(c, stage_id, len);
    HIPC(c, hipMemcpyAsync(c->pin + kPinSmall, d_fin, sizeof(State), hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipEventRecord(c->ev_fin, c->stream));
    return MSA_OK;
}
static int wait_scan_fn(msa_ctx *c, State *fin) {
    if (!c->fin_pending) {
        *fin = c->fin_init;
        return MSA_OK;
    }
    c->fin_pending = false;
    HIPC(c, hipEventSynchronize(c->ev_fin));
    memcpy(fin, c->pin + kPinSmall, sizeof(State));
    return MSA_OK;
}
static int run_scan_fn(msa_ctx *c, const u8 *buf, u64 b, u64 e, State init, State *fin, int stage_id) {
    int rc;
    if ((rc = launch_scan_fn(c, buf, b, e, init, stage_id))) return rc;
    return wait_scan_fn(c, fin);
}

static u32 log2_ceil(u64 v) {
    u32 k = 0;
    while ((1ull << k) < v) ++k;
    return k;
}

static int ensure_tables(msa_ctx *c) {
    // Tables are zeroed once at allocation; after each run only the claimed
    // slots are cleared again (no per-run memset of a whole table).
    const u64 n = c->n;
    // distinct keys can never exceed tokens (<= n/4) / records: cap the growth there
    const u32 cap_s = std::max<u32>(16, log2_ceil(n / 2 + 1));
    if (!c->s_log2) c->s_log2 = std::min<u32>(20, cap_s);
    if (!c->m_log2) c->m_log2 = std::min<u32>(18, cap_s);
    if (!c->lt_log2) c->lt_log2 = std::min<u32>(16, cap_s);
    // long-word positions: a word of > 16 bytes and its separator take >= 18
    // bytes; room for one in every 128 bytes (20 B of arrays per slot) covers
    // corpora far richer in long words than lyrics without a retry -- a cold run
    // had repeated its whole split for them (configs[4])
    if (!c->l_occ_want) c->l_occ_want = std::max<u64>(1ull << 16, n / 128);
    const u32 a_need = log2_ceil(std::max<u64>(1ull << 12, 2 * (c->nrec + 1)));
    if (!c->a_log2) c->a_log2 = std::min<u32>(16, a_need);
    const u64 s_slots = 1ull << c->s_log2, m_slots = 1ull << c->m_log2, lt_slots = 1ull << c->lt_log2;
    const u64 a_slots = 1ull << c->a_log2;
    const u64 l_occ = c->l_occ_want;
    if (s_slots != c->s_slots) {
        release(c->s_tab);
        HIPC(c, ensure(c->s_tab, s_slots * 16, true));
        HIPC(c, ensure(c->s_list, (s_slots / 2) * 4));
        c->s_slots = s_slots;
        c->s_used_prev = 0;
    }
    if (m_slots != c->m_slots) {
        release(c->m_tab);
        HIPC(c, ensure(c->m_tab, m_slots * 32, true));
        HIPC(c, ensure(c->m_list, (m_slots / 2) * 4));
        c->m_slots = m_slots;
        c->m_used_prev = 0;
    }
    if (l_occ != c->l_occ_cap) {
        HIPC(c, ensure(c->l_pos, l_occ * 8));
        HIPC(c, ensure(c->l_len, l_occ * 4));
        HIPC(c, ensure(c->l_slot, l_occ * 8));
        c->l_occ_cap = l_occ;
    }
    if (lt_slots != c->lt_slots) {
        release(c->l_tab);
        HIPC(c, ensure(c->l_tab, lt_slots * 32, true));
        HIPC(c, ensure(c->l_list, (lt_slots / 2) * 4));
        c->lt_slots = lt_slots;
        c->lt_used_prev = 0;
    }
    if (a_slots != c->a_slots) {
        release(c->a_tab);
        HIPC(c, ensure(c->a_tab, a_slots * 32, true));
        HIPC(c, ensure(c->a_list, (a_slots / 2) * 4));
        c->a_slots = a_slots;
        c->a_used_prev = 0;
    }
    return MSA_OK;
}

// After an overflow: grow exactly the tables that overflowed, to at least
// twice what the failed run claimed (claim counters keep counting past the
// list capacity), and at least 8x.  `mask` selects the overflow bits of the
// stage that is retried.
static void grow_tables(msa_ctx *c, u64 mask = ~0ull) {
    const u64 f = c->h_ctr.overflow & mask;
    // a grown table has >= 4 slots per key the failed run claimed and at
    // least 8 times the slots it had (2 slots per key in one step measured: no
    // change)
    constexpr u64 mul = 4;
    constexpr u32 step = 3;
    auto grow = [](u32 &lg, u64 claimed) {
        const u32 want = log2_ceil(std::max<u64>(claimed * mul, 1));
        lg = std::max<u32>(lg + step, want);
        if (lg > 31) lg = 31;  // slot lists hold u32 indices
    };
    if (f & OVF_S) grow(c->s_log2, c->h_ctr.s_claimed);
    if (f & OVF_M) grow(c->m_log2, c->h_ctr.m_claimed);
    if (f & OVF_LT) grow(c->lt_log2, c->h_ctr.l_claimed);
    if (f & OVF_A) {  // artists <= records: one step to the size that holds any input of this length
        grow(c->a_log2, c->h_ctr.a_claimed);
        const u32 a_need = log2_ceil(std::max<u64>(1ull << 12, 2 * (c->nrec + 1)));
        if (c->a_log2 < a_need && a_need <= 31) c->a_log2 = a_need;
    }
    if (f & OVF_L) c->l_occ_want = std::max<u64>(c->l_occ_want * 8, c->h_ctr.l_occ * 2);
}

// clear only the slots the previous run claimed
__global__ void k_clear_slots(u64 *tab, const u32 *list, u64 n, u32 words_per_slot) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    u64 *s = tab + (u64)list[i] * words_per_slot;
    for (u32 k = 0; k < words_per_slot; ++k) s[k] = 0;
}

// Every read-back of the run counters also settles the column lengths the
// split left on the device.
static void take_col_lens(msa_ctx *c) {
    if (!c->col_lens_pending) return;
    c->acol_len = c->col_hdr[0] + c->h_ctr.col_body[0];
    c->tcol_len = c->have_tcol ? c->col_hdr[1] + c->h_ctr.col_body[1] : 0;
    c->a_end = c->acol_len;
    c->col_lens_pending = false;
    // text.csv's stage bytes, now that the body length is known: the body read
    // and written + per record its span (len, offset, source, "" pairs: 28 B)
    if (c->ps[ST_TEXT_COLUMN].pending && c->have_tcol)
        c->ps[ST_TEXT_COLUMN].pend_bytes = 2 * c->h_ctr.col_body[1] + c->nrec * 28;
}
static int sync_counters(msa_ctx *c) {
    HIPC(c, hipMemcpyAsync(c->pin, c->ctr.p, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    memcpy(&c->h_ctr, c->pin, sizeof(Counters));
    take_col_lens(c);
    return MSA_OK;
}
static int resolve_col_lens(msa_ctx *c) { return c->col_lens_pending ? sync_counters(c) : MSA_OK; }

// After a failed (overflowed) attempt the tables hold partial counts and their
// slot lists may be incomplete: zero the whole tables instead of the claimed
// slots (rare path).
static int wipe_tables(msa_ctx *c) {
    struct {
        DevBuf *tab;
        u64 slots, *used;
        u32 w;
    } t[4] = {{&c->s_tab, c->s_slots, &c->s_used_prev, 2},
              {&c->m_tab, c->m_slots, &c->m_used_prev, 4},
              {&c->l_tab, c->lt_slots, &c->lt_used_prev, 4},
              {&c->a_tab, c->a_slots, &c->a_used_prev, 4}};
    for (auto &x : t) {
        if (x.tab->p && x.slots) HIPC(c, hipMemsetAsync(x.tab->p, 0, x.slots * x.w * 8, c->stream));
        *x.used = 0;
    }
    return MSA_OK;
}
static int wipe_one(msa_ctx *c, DevBuf &tab, u64 slots, u32 w, u64 &used) {
    if (tab.p && slots) HIPC(c, hipMemsetAsync(tab.p, 0, slots * w * 8, c->stream));
    used = 0;
    return MSA_OK;
}
// Zero counter fields on the stream (a stage about to be retried).
static int reset_ctr(msa_ctx *c, u64 Counters::*f) {
    Counters *dc = c->ctr.as<Counters>();
    HIPC(c, hipMemsetAsync(&(dc->*f), 0, 8, c->stream));
    return MSA_OK;
}
// Fresh artist table (grown or not) and its counters, for a repeated keying.
static int ensure_tables(msa_ctx *c);
static int reset_artist_table(msa_ctx *c) {
    int rc;
    if ((rc = ensure_tables(c))) return rc;
    if ((rc = wipe_one(c, c->a_tab, c->a_slots, 4, c->a_used_prev))) return rc;
    c->a_dirty = false;
    if ((rc = reset_ctr(c, &Counters::a_claimed))) return rc;
    if ((rc = reset_ctr(c, &Counters::overflow))) return rc;
    if ((rc = reset_ctr(c, &Counters::songs))) return rc;  // the lines kernel counts them again
    return reset_ctr(c, &Counters::collision);
}

// ------------------------------------------------------------------ stage 1
// The column's length stays on the device (no host round trip): every line is
// at most as long as its record, so header + input bytes bound the column;
// the length lands in Counters::col_body[text] and reaches the host with the
// next counter read-back (col_lens_pending).
// Line offsets of both columns: one scan launch sequence over both length
// arrays (the bodies' totals stay on the device, Counters::col_body).
static int scan_columns(msa_ctx *c, bool text, hipStream_t st) {
    const u64 nrec = c->nrec;
    const u64 nbb = (nrec + 1023) / 1024 + 1;
    HIPC(c, ensure(c->aoff, nrec * 8));
    if (text) HIPC(c, ensure(c->toff, nrec * 8));
    HIPC(c, ensure(c->scan_bsum, 2 * nbb * 8));
    u64 *body = c->ctr.as<Counters>()->col_body;
    u64 *bs = c->scan_bsum.as<u64>();
    HIPC(c, msa_exclusive_scan2(c->alen.as<u64>(), nrec, c->aoff.as<u64>(), bs, &body[0],
                                text ? c->tlen.as<u64>() : nullptr, nrec, c->toff.as<u64>(), bs + nbb, &body[1],
                                st));
    return MSA_OK;
}

// A column's body at col + hdr (its header line is written by put_bytes).
static int materialise_column(msa_ctx *c, bool text, u64 hdr, DevBuf &col, DevBuf &lenb, DevBuf &offb,
                              DevBuf &srcb, DevBuf &pairsb, hipStream_t st) {
    const u64 nrec = c->nrec;
    u64 *body_p = &c->ctr.as<Counters>()->col_body[text ? 1 : 0];  // from scan_columns
    // the artist column reads lines equal to their keys from the arena k_rec_fast filled
    const bool keys = !text && c->spans;
    HIPC(c, msa_launch_col_write(text ? 1 : 0, c->in, lenb.as<u64>(), offb.as<u64>(), srcb.as<u64>(), pairsb.as<u32>(),
                                 nrec, hdr, body_p, col.as<u8>(), keys ? c->arena.as<u8>() : nullptr,
                                 c->key_off.as<u64>(), c->key_len.as<u32>(), st));
    return MSA_OK;
}

// Small host values written by a kernel (a pageable hipMemcpyAsync source
// makes the call wait for the stream to drain up to the copy).
struct Bytes256 {
    unsigned char b[256];
};
__global__ void k_put_bytes(u8 *dst, Bytes256 v, u32 n) {
    if (threadIdx.x < n) dst[threadIdx.x] = v.b[threadIdx.x];
}
// The deferred body of text.csv on stream st (the side stream: after what is
// enqueued on the library stream so far).
static int launch_text(msa_ctx *c, hipStream_t st) {
    int rc;
    c->text_deferred = false;
    prof_begin(c, ST_TEXT_COLUMN, st);
    if ((rc = materialise_column(c, true, kColHdrRoom, c->tcol, c->tlen, c->toff, c->tsrc, c->tpairs, st))) return rc;
    prof_end(c, ST_TEXT_COLUMN, c->n * 2 + c->nrec * 40, st);  // ~ the text column read + written
    return MSA_OK;
}
static int start_text_side(msa_ctx *c) {
    if (!c->text_deferred) return MSA_OK;
    int rc;
    HIPC(c, fork_side(c));
    if ((rc = launch_text(c, c->side))) return rc;
    HIPC(c, hipEventRecord(c->ev_join, c->side));
    c->side_pending = true;
    return MSA_OK;
}
static int put_bytes(msa_ctx *c, u8 *dst, const std::string &b, hipStream_t st) {
    if (b.empty()) return MSA_OK;
    if (b.size() > sizeof(Bytes256)) return fail(c, MSA_ERR_ARG, "header line longer than %zu bytes", sizeof(Bytes256));
    Bytes256 v;
    memcpy(v.b, b.data(), b.size());
    hipLaunchKernelGGL(k_put_bytes, dim3(1), dim3(256), 0, st, dst, v, (u32)b.size());
    HIPC(c, hipGetLastError());
    return MSA_OK;
}
__global__ void k_put_u64(u64 *p0, u64 v0, u64 *p1, u64 v1) {
    if (threadIdx.x == 0 && p0) *p0 = v0;
    if (threadIdx.x == 1 && p1) *p1 = v1;
}

// The main scan inserts into the HBM word tables without appending to their
// slot lists; the lists and claimed counts are built here, once per table.
static int build_word_lists(msa_ctx *c, hipStream_t st = nullptr) {
    Counters *dc = c->ctr.as<Counters>();
    if (!st) st = c->stream;
    HIPC(c, msa_launch_list_build(c->s_tab.as<u64>(), c->s_slots, 2, c->s_list.as<u32>(), c->s_slots / 2,
                                  &dc->s_claimed, dc, (u64)OVF_S, st));
    HIPC(c, msa_launch_list_build(c->m_tab.as<u64>(), c->m_slots, 4, c->m_list.as<u32>(), c->m_slots / 2,
                                  &dc->m_claimed, dc, (u64)OVF_M, st));
    return MSA_OK;
}

// Column materialisation after the scan.  ah / th are the header lines of
// artist.csv / text.csv (empty for a continuation shard).
// Line spans of both columns and the artist keys, then the offset scans: they
// depend on the scan alone, so they are enqueued before its read-back (the
// host's header work overlaps them).
static int launch_spans(msa_ctx *c, bool want_text, hipStream_t st) {
    int rc;
    prof_begin(c, ST_REC_SPANS, st);
    const u64 nrec = c->nrec;
    HIPC(c, ensure(c->alen, nrec * 8));
    HIPC(c, ensure(c->asrc, nrec * 8));
    HIPC(c, ensure(c->apairs, nrec * 4));
    if (want_text) {
        HIPC(c, ensure(c->tlen, nrec * 8));
        HIPC(c, ensure(c->tsrc, nrec * 8));
        HIPC(c, ensure(c->tpairs, nrec * 4));
    }
    // artist keys for the lines shortcut of the artist pass (msa_count)
    if (!c->a_long_cap) c->a_long_cap = std::max<u64>(1ull << 20, c->n / 32);
    const u64 long_base = 32 * (nrec + 2);
    HIPC(c, ensure(c->arena, long_base + c->a_long_cap + 64));  // + 64: 16-byte loads past a key's end
    HIPC(c, ensure(c->key_off, (nrec + 2) * 8));
    HIPC(c, ensure(c->key_len, (nrec + 2) * 4));
    HIPC(c, ensure(c->kh1, (nrec + 2) * 8));
    HIPC(c, ensure(c->kh2, (nrec + 2) * 8));
    AKeys ak{c->arena.as<u8>(), c->key_off.as<u64>(), c->key_len.as<u32>(), c->kh1.as<u64>(), c->kh2.as<u64>(),
             long_base, c->a_long_cap};
    if (c->spans) HIPC(c, ensure(c->span_fix, (nrec + 1) * 8));
    // k_rec_fast's own stage: per record 32 B of span events read (rec_start,
    // f0, tss, tse), the record's first 32 bytes (its artist key), and 100 B
    // written (both columns' len / src / pairs 40, key off / len / two
    // hashes 28, the 32-byte key arena slot)
    prof_begin(c, ST_REC_FAST, st);
    const hipEvent_t fast_end = prof_end_event(c, ST_REC_FAST, nrec * 164);
    HIPC(c, msa_launch_rec_spans(c->in, c->rec_start.as<u64>(), c->nulrel.as<u32>(), nrec, c->cont ? 0 : 1,
                                 want_text ? 1 : 0, c->alen.as<u64>(), c->asrc.as<u64>(), c->apairs.as<u32>(),
                                 c->tlen.as<u64>(), c->tsrc.as<u64>(), c->tpairs.as<u32>(), c->ctr.as<Counters>(), ak,
                                 c->spans ? c->f0.as<u64>() : nullptr, c->tss.as<u64>(), c->tse.as<u64>(),
                                 c->span_fix.as<u64>(), c->ablate, st, fast_end));
    if (st == c->rank2) HIPC(c, hipEventRecord(c->ev_fix, st));  // the artist pass may start here
    if ((rc = scan_columns(c, want_text, st))) return rc;
    prof_end(c, ST_REC_SPANS, nrec * 136, st);  // ~36 B read + 100 B written per record
    return MSA_OK;
}

static int split_columns_rest(msa_ctx *c, bool want_text, const std::string &ah, const std::string &th) {
    HIPC(c, ensure(c->acol, ah.size() + c->n + 1 + MSA_INPUT_PAD));
    c->artist_hdr = ah;  // deferred (see msa_ctx::artist_deferred)
    c->artist_deferred = true;
    // compute_header_length (parallel_spotify.c:444-459): getline's end
    c->a_hdr_getline = ah.empty() ? 0 : ah.find('\n') + 1;
    c->a_hdr_len = ah.size();
    c->a_beg = c->a_hdr_getline;
    c->col_hdr[0] = ah.size();
    c->col_hdr[1] = th.size();
    c->col_lens_pending = true;  // acol_len / tcol_len / a_end: from the next counter read-back
    c->have_tcol = false;
    if (want_text) {  // the body is on its way (start_text_side): the header line goes right before it
        if (th.size() > kColHdrRoom) return fail(c, MSA_ERR_ARG, "text header line longer than %llu bytes",
                                                 (unsigned long long)kColHdrRoom);
        c->tcol_off = kColHdrRoom - th.size();
        int rc;
        if ((rc = put_bytes(c, c->tcol.as<u8>() + c->tcol_off, th, c->stream))) return rc;
        c->have_tcol = true;
    }
    c->stage = 1;
    return MSA_OK;
}

// The S/M slots a split claimed (cleared by the next split's prologue); a
// dense split claims none.
static void set_used_prev(msa_ctx *c) {
    c->s_used_prev = c->dense_w ? 0 : std::min<u64>(c->h_ctr.s_claimed, c->s_slots / 2);
    c->m_used_prev = c->dense_w ? 0 : std::min<u64>(c->h_ctr.m_claimed, c->m_slots / 2);
}
// Word-table overflows of the scan (S/M tables, long-word occurrence list):
// the split is repeated with grown tables (msa_split_columns' retry loop).
// OVF_MLOG: K3 dropped misses (logs grown); OVF_DENSE: a dense split's retry
static const u64 kSplitOvf = OVF_S | OVF_M | OVF_L | OVF_MLOG | OVF_DENSE;
static int check_split_overflow(msa_ctx *c, bool read_back = true) {
    int rc;
    if (read_back && (rc = sync_counters(c))) return rc;
    if (c->h_ctr.overflow & OVF_FOLD)
        return fail(c, MSA_ERR_HIP, "split scan: a tile's look-back timed out");
    if (c->h_ctr.overflow & kSplitOvf)
        return fail(c, MSA_ERR_CAPACITY, "word table capacity overflow (flags 0x%llx)",
                    (unsigned long long)c->h_ctr.overflow);
    // the S/M slots this split claimed: the next split clears them even when no
    // msa_count ran in between
    set_used_prev(c);
    return MSA_OK;
}

// Before the split's K1, in one launch: the claimed slots of the four tables
// cleared, the run counters zeroed, nulrel[0, nul_n) zeroed, rec_start[0] = 0
// (four clear launches, a memset and two copies before: ~60 us of launch gaps).
struct ClearJob {
    u64 *tab;
    const u32 *list;
    u64 n;
    u32 w, blocks;
};
struct Prologue {
    ClearJob job[4];
    u64 *ctr;
    u32 ctr_words, fill_blocks;
    u32 *nul;
    u64 nul_n;
    u64 *rs0;
};
#define PRO_T 256
__global__ __launch_bounds__(PRO_T) void k_prologue(Prologue p) {
    u32 b = blockIdx.x;
    const u32 t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (b < p.job[j].blocks) {
            const u64 i = (u64)b * PRO_T + t;
            if (i < p.job[j].n) {
                u64 *s = p.job[j].tab + (u64)p.job[j].list[i] * p.job[j].w;
                for (u32 k = 0; k < p.job[j].w; ++k) s[k] = 0;
            }
            return;
        }
        b -= p.job[j].blocks;
    }
    if (b == 0) {
        if (t < p.ctr_words) p.ctr[t] = 0;
        if (t == 0 && p.rs0) *p.rs0 = 0;
        for (u64 i = (p.nul_n & ~3ull) + t; i < p.nul_n; i += PRO_T) p.nul[i] = 0;
    }
    uint4 *q = reinterpret_cast<uint4 *>(p.nul);
    for (u64 i = (u64)b * PRO_T + t; i < p.nul_n / 4; i += (u64)p.fill_blocks * PRO_T) q[i] = make_uint4(0, 0, 0, 0);
}
static int split_prologue(msa_ctx *c, u64 nul_n, bool rs0) {
    Prologue p{};
    struct {
        DevBuf *tab, *list;
        u64 *used, slots;
        u32 w;
    } t[4] = {{&c->s_tab, &c->s_list, &c->s_used_prev, c->s_slots, 2},
              {&c->m_tab, &c->m_list, &c->m_used_prev, c->m_slots, 4},
              {&c->l_tab, &c->l_list, &c->lt_used_prev, c->lt_slots, 4},
              {&c->a_tab, &c->a_list, &c->a_used_prev, c->a_slots, 4}};
    u32 blocks = 0;
    for (int j = 0; j < 4; ++j) {
        u64 n = t[j].tab->p ? *t[j].used : 0;
        // a slot cleared by itself costs about as much as zeroing 256 bytes
        // of a whole table (configs[4]: 18.5 M claimed 9..16-byte word slots
        // took 0.9 ms of scattered clears, a 4 GiB table 0.6 ms of memset):
        // past that, the table is zeroed whole
        if (n && n * 256 > t[j].slots * t[j].w * 8 && !(c->ablate & 1048576)) {
            HIPC(c, hipMemsetAsync(t[j].tab->p, 0, t[j].slots * t[j].w * 8, c->stream));
            n = 0;
        }
        p.job[j] = ClearJob{t[j].tab->as<u64>(), t[j].list->as<u32>(), n, t[j].w, (u32)((n + PRO_T - 1) / PRO_T)};
        blocks += p.job[j].blocks;
        *t[j].used = 0;
    }
    static_assert(sizeof(Counters) % 8 == 0 && sizeof(Counters) / 8 <= PRO_T, "k_prologue zeroes Counters in one block");
    p.ctr = c->ctr.as<u64>();
    p.ctr_words = sizeof(Counters) / 8;
    p.nul = c->nulrel.as<u32>();
    p.nul_n = nul_n;
    p.rs0 = rs0 ? c->rec_start.as<u64>() : nullptr;
    p.fill_blocks = (u32)std::min<u64>(1024, std::max<u64>(1, (nul_n / 4 + PRO_T - 1) / PRO_T));
    hipLaunchKernelGGL(k_prologue, dim3(blocks + p.fill_blocks), dim3(PRO_T), 0, c->stream, p);
    HIPC(c, hipGetLastError());
    return MSA_OK;
}

static int launch_artist_count(msa_ctx *c, hipStream_t st = nullptr);
static int split_once(msa_ctx *c, int flags) {
    int rc;
    c->artist_deferred = c->text_deferred = false;  // superseded by this split
    HIPC(c, join_side(c));  // a text column pass in flight reads buffers this one rewrites
    if (!c->in) return fail(c, MSA_ERR_ARG, "no input bound (msa_load_csv / msa_bind_csv)");
    if (c->n == 0 && !c->cont) return fail(c, MSA_ERR_NOHEADER, "Dataset does not contain a header row");
    const bool want_text = (flags & MSA_SPLIT_TEXT_COLUMN) != 0;
    c->merged_w = c->merged_a = false;
    c->ranked_only = 0;
    c->artist_piece_set = false;
    c->artist_spec = false;
    c->col_lens_pending = false;
    c->extra_len = 0;
    HIPC(c, ensure(c->ctr, sizeof(Counters)));
    // K3 is launched right behind K2 on the record arrays an earlier split
    // sized (cap0 records), and checked against K2's record count when the
    // host reads it back -- K3 runs meanwhile.  Too small (the first split, or
    // a larger input): the arrays grow and K3 runs again.
    u64 cap0 = c->rec_cap;
    if (c->fold && !cap0 && c->n) {
        // the folded scan learns the record count as it writes the records: the
        // first split guesses (a record per 64 bytes) and runs again if short
        const u64 g = std::max<u64>(1024, c->n / 64) + 2;
        HIPC(c, ensure(c->rec_start, g * 8));
        HIPC(c, ensure(c->nulrel, g * 4));
        HIPC(c, ensure(c->f0, g * 8));
        HIPC(c, ensure(c->tss, g * 8));
        HIPC(c, ensure(c->tse, g * 8));
        c->rec_cap = cap0 = g;
    }
    if (c->a_dirty) {  // an earlier split's artist count overflowed and no msa_count wiped the table
        if ((rc = ensure_tables(c)) || (rc = wipe_one(c, c->a_tab, c->a_slots, 4, c->a_used_prev))) return rc;
        c->a_dirty = false;
    }
    if ((rc = split_prologue(c, want_text ? cap0 : 0, cap0 != 0))) return rc;
    State init{0, 0, 0, 0, 0, 0}, fin;
    if (c->fold) {
        // K1 + K2 folded into the structure pass (launch_k3; the status words
        // pack record indices in 40 bits: inputs < 1 TiB, HBM holds 288 GB)
        if (c->n >= (1ull << 40)) return fail(c, MSA_ERR_ARG, "input of %llu bytes: 1 TiB or more", (unsigned long long)c->n);
        c->fin_init = init;
        c->fin_pending = false;
    } else if ((c->ablate & 16384) && c->fin_cache_n == c->n + 1) {
        // diagnostic (MSA_ABLATE bit 16384, valid only for an unchanged input):
        // K1 + K2 skipped, the chunk states of the previous split reused -- the
        // ceiling of what folding K1 into the record pass could save
        c->fin_init = c->fin_cache;
        c->fin_pending = false;
    } else if ((rc = launch_scan_fn(c, c->in, 0, c->n, init, ST_CSV_SUMMARY))) {
        return rc;
    }

    ScanArgs a{};
    auto launch_k3 = [&](u64 cap) -> int {
        if ((rc = ensure_tables(c))) return rc;
        a = ScanArgs{};
        a.buf = c->in;
        a.seg_begin = 0;
        a.seg_end = c->n;
        a.nchunks = (u32)((c->n + MSA_CHUNK - 1) / MSA_CHUNK);
        a.carry = c->carry.as<State>();
        a.sums = c->sums.as<ChunkSum>();  // from launch_scan_fn over the same [0, n)
        a.rec_start = c->rec_start.as<u64>();
        a.nulrel = c->nulrel.as<u32>();
        a.rec_cap = cap;
        a.f0 = c->f0.as<u64>();
        a.tss = c->tss.as<u64>();
        a.tse = c->tse.as<u64>();
        c->spans = true;
        a.s_tab = c->s_tab.as<u64>();
        a.s_mask = c->s_slots - 1;
        a.s_list = c->s_list.as<u32>();
        a.s_list_cap = c->s_slots / 2;
        a.m_tab = c->m_tab.as<u64>();
        a.m_mask = c->m_slots - 1;
        a.m_list = c->m_list.as<u32>();
        a.m_list_cap = c->m_slots / 2;
        a.l_pos = c->l_pos.as<u64>();
        a.l_cap = c->l_occ_cap;
        a.l_expect = c->l_occ_last ? c->l_occ_last : c->n / 1024;
        a.ctr = c->ctr.as<Counters>();
        a.want_nul = want_text ? 1 : 0;
        a.ablate = c->ablate;
        a.first_rec = c->cont ? 0 : 1;
        {  // miss logs: room for about a quarter of the tokens, or for what the last
           // split logged (a full partition drops its further entries and flags
           // OVF_MLOG: the split runs again with larger logs; past the 2^24-entry
           // partition limit the token pass inserts them into HBM instead)
            const u64 parts = (u64)c->cus * msa_tok_wgcu() * MSA_MLOG_PARTS;
            u64 entries = std::max<u64>(std::max<u64>(parts * 1024, c->n / 16), c->mlog_want);
            if (c->mlog_test) entries = std::max<u64>(c->mlog_test, c->mlog_want);  // tests: small first logs
            // (a workgroup's 16 partitions are addressed with 32-bit byte offsets)
            a.mlog_cap = (u32)std::min<u64>(entries / parts, (1u << 24) - 1);
            a.mlog_direct = entries / parts > a.mlog_cap;  // growing them further is impossible
            c->mlog_cap_last = a.mlog_cap;
            HIPC(c, ensure(c->mlog, parts * a.mlog_cap * 16));
            HIPC(c, ensure(c->mlog_n, parts * 4));
            a.mlog = c->mlog.as<ulonglong2>();
            a.mlog_n = c->mlog_n.as<u32>();
        }
        {  // a word per 64 bytes of every 4 KiB block, behind one zero word
            const u64 words = (c->n + 4095) / 4096 * 64 + 2;
            if (c->lmask.cap < words * 8) {
                HIPC(c, ensure(c->lmask, words * 8));
                HIPC(c, hipMemsetAsync(c->lmask.p, 0, 8, c->stream));
            }
            a.lmask = c->lmask.as<u64>();
        }
        prof_begin(c, ST_CSV_SCAN);
        if (c->fold) {  // k_scan_fold: K1 + K2 + k_scan_struct in one pass
            const u32 ntiles = msa_fold_tiles(a.nchunks);
            const u64 need = 8 + (u64)ntiles * 5 * 8;
            if (c->fold_buf.cap < need) {  // new statuses: zeroed, epochs start over
                HIPC(c, ensure(c->fold_buf, need, true));
                c->fold_tbase = 0;
                c->fold_ep = 0;
            }
            if (++c->fold_ep == 0x10000) {  // the epoch wraps: no stale status may match
                HIPC(c, hipMemsetAsync(c->fold_buf.as<u64>() + 1, 0, c->fold_buf.cap - 8, c->stream));
                c->fold_ep = 1;
            }
            a.fold_ticket = c->fold_buf.as<u64>();
            a.fold_stat = a.fold_ticket + 1;
            a.fold_n = (u32)((c->fold_buf.cap - 8) / 40);
            a.fold_tbase = c->fold_tbase;
            a.fold_ep = c->fold_ep;
            a.fold_init = State{0, 0, 0, 0, 0, 0};
            HIPC(c, ensure(c->small, 4096));
            a.fold_fin = reinterpret_cast<State *>(c->small.as<char>() + 1024);
            a.fold_fin_host = reinterpret_cast<State *>(c->pin + kPinSmall);
            u64 tickets = 0;
            HIPC(c, msa_launch_scan_fold(a, &tickets, c->stream));
            c->fold_tbase += tickets;
            HIPC(c, hipEventRecord(c->ev_fin, c->stream));  // the kernel wrote the final state to c->pin
            c->fin_pending = a.nchunks != 0;
            c->fin_init = a.fold_init;
        } else {
            HIPC(c, msa_launch_scan_csv(a, c->stream));  // k_scan_struct (msa_k3.hip)
        }
        // algorithmic bytes: every CSV byte once + the per-record SoA it writes
        // (rec_start 8, nulrel 4 with the text column, the span events f0 / tss / tse 24)
        // + the split scan's token-byte mask (1 bit per byte)
        prof_end(c, ST_CSV_SCAN, c->n + c->nrec * ((want_text ? 12ull : 8ull) + 24ull) + c->n / 8);
        {
            HIPC(c, hipEventRecord(c->ev_scan_a, c->stream));  // the record arrays are final
            prof_begin(c, ST_CSV_TOKENS);
            HIPC(c, msa_launch_scan_tokens(a, c->stream));
            // the mask (1 bit per byte) + the token bytes re-read (at most every byte once)
            prof_end(c, ST_CSV_TOKENS, c->n + c->n / 8);
        }
        return MSA_OK;
    };
    if (cap0 && (rc = launch_k3(cap0))) return rc;
    if ((rc = wait_scan_fn(c, &fin))) return rc;
    c->fin_cache = fin;
    c->fin_cache_n = c->n + 1;
    const u64 nterm = fin.rec;
    c->nrec = nterm + (fin.rs < c->n ? 1 : 0);
    const u64 cap = nterm + 2;
    if (cap > cap0) {
        if (cap0) {  // K3 ran out of record room: its counts are undone, it runs again
            HIPC(c, hipStreamSynchronize(c->stream));
            if ((rc = wipe_tables(c))) return rc;
            HIPC(c, hipMemsetAsync(c->ctr.p, 0, sizeof(Counters), c->stream));
        }
        HIPC(c, ensure(c->rec_start, cap * 8));
        HIPC(c, ensure(c->nulrel, cap * 4));
        HIPC(c, ensure(c->f0, cap * 8));
        HIPC(c, ensure(c->tss, cap * 8));
        HIPC(c, ensure(c->tse, cap * 8));
        c->rec_cap = cap;
        if (want_text) HIPC(c, hipMemsetAsync(c->nulrel.p, 0, cap * 4, c->stream));
        HIPC(c, hipMemsetAsync(c->rec_start.p, 0, 8, c->stream));
        if ((rc = launch_k3(cap))) return rc;
        c->fin_pending = false;  // the folded scan's state again: known
    }
    // The column spans depend on the record arrays alone: with the split scan
    // they run on the rank2 stream from the end of k_scan_struct, beside
    // k_scan_tokens (whose one workgroup per CU leaves wave slots free) and
    // k_miss_agg.  (The fused scan: k_miss_agg measured beside k_rec_fast on
    // rank2 -- both kernels took twice as long, no gain.)
    const bool spans_beside = !(c->ablate & 8192);
    hipStream_t sst = c->stream;
    if (spans_beside) {
        sst = c->rank2;
        HIPC(c, hipStreamWaitEvent(c->rank2, c->ev_scan_a, 0));
    }
    // the context's first split of a large input has no count to go by: it
    // takes the dense entries, exact at any cardinality, and later splits
    // choose by its count -- a table split that overflowed had cost a cold
    // configs[4] run a 0.12 s aggregation into full tables before its repeat
    // (a wrong guess costs a low-cardinality input ~1 ms once)
    const bool cold_big = !c->have_hist && c->n >= (64ull << 20);
    c->dense_w = c->dense_on && !c->dense_veto && !a.mlog_direct &&
                 (c->prev_distinct >= c->dense_min || cold_big);
    if (c->dense_w) {
        // the words' entry planes, written by the bucketed aggregation: room
        // for every logged entry a distinct key, plus the long words
        // (k_word_entries appends them in msa_rank)
        Ranked &W = c->rw;
        const u64 cap = (u64)msa_scan_blocks(a) * MSA_MLOG_PARTS * a.mlog_cap;
        const u64 n = cap + c->lt_slots / 2 + 1;
        for (int k = 0; k < 3; ++k) HIPC(c, ensure(W.K[0][k], n * 8));
        HIPC(c, ensure(W.V[0], n * 4));
        HIPC(c, ensure(W.ref, n * 8));
        HIPC(c, ensure(W.cnt, n * 8));
        HIPC(c, ensure(W.vary, msa_dn_vary_words() * 8));
        a.dn_K2 = W.K[0][0].as<u64>();
        a.dn_K1 = W.K[0][1].as<u64>();
        a.dn_K0 = W.K[0][2].as<u64>();
        a.dn_val = W.V[0].as<u32>();
        a.dn_ref = W.ref.as<u64>();
        a.dn_cnt = W.cnt.as<u64>();
        a.dn_vary = W.vary.as<u64>();
        a.dn_cap = cap;
    }
    {
        prof_begin(c, ST_MISS_AGG);
        // high cardinality (the last split's logs held far more distinct keys
        // than the aggregating workgroups' LDS tables): bucketed first
        const bool mb = c->dense_w || c->mb_mode == 1 || (c->mb_mode == 2 && c->mb_prev > c->mb_min);
        if (mb) {
            const u64 hw = msa_mb_hist_words(a, msa_scan_blocks(a));
            HIPC(c, ensure(c->mb_hist, hw * 8));
            HIPC(c, ensure(c->mb_off, hw * 8));
            HIPC(c, ensure(c->mb_bsum, ((hw + 1023) / 1024 + 1) * 8));
            HIPC(c, ensure(c->mb_tot, 64));
            HIPC(c, ensure(c->mb_out, (u64)msa_scan_blocks(a) * MSA_MLOG_PARTS * a.mlog_cap * 16));
            HIPC(c, msa_launch_miss_buckets(a, c->mb_hist.as<u64>(), c->mb_off.as<u64>(), c->mb_bsum.as<u64>(),
                                            c->mb_tot.as<u64>(), c->mb_out.as<ulonglong2>(), c->stream));
        } else {
            HIPC(c, msa_launch_miss_agg(a, c->stream));
        }
        prof_end(c, ST_MISS_AGG, 0);
    }
    // rec_start[nrec] = end of the last record (EOF when it has no terminator);
    // no terminator: k_rec_fast leaves the last record to the exact path
    if (fin.rs < c->n) {
        hipLaunchKernelGGL(k_put_u64, dim3(1), dim3(64), 0, sst, c->rec_start.as<u64>() + c->nrec, (u64)c->n,
                           c->tse.as<u64>() + c->nrec - 1, (u64)SPAN_FIX);
        HIPC(c, hipGetLastError());
    }
    if ((rc = launch_spans(c, want_text, sst))) return rc;
    if (spans_beside) {
        HIPC(c, hipEventRecord(c->ev_spans, c->rank2));
#if !MSA_LISTS_BEFORE_SPANS
        HIPC(c, hipStreamWaitEvent(c->stream, c->ev_spans, 0));
#endif
    }
    if (want_text) {  // text.csv's body: deferred (msa_ctx::text_deferred)
        HIPC(c, ensure(c->tcol, kColHdrRoom + c->n + 1 + MSA_INPUT_PAD));
        c->text_deferred = true;
    }
    // one read-back after the scan: the counters (table overflow, long-word
    // occurrences) and -- for the first shard -- the header record's end plus
    // the input's first bytes (the header, almost always)
    // the word tables' slot lists (table scans: streaming) on rank2 beside the
    // artist pass (LDS tables and atomics) -- both only add to Counters with
    // atomics; the read-back below waits for both
    // (measured neutral on rank2 beside the artist pass, profiles/r04_t41_*)
    const bool art_ok = !c->artist_exact && c->nrec && !(c->ablate & 32768);
#if MSA_ARTIST_SIDE && MSA_LISTS_BEFORE_SPANS && MSA_ARTIST_EARLY
    // with text.csv: the artist pass and then text.csv's gather on the side
    // stream, from rank2's k_rec_fix (the keys) and its offset scans -- not
    // from the library stream, whose k_miss_agg and slot lists they do not
    // need (the table clears of the prologue came before rank2's fork).  The
    // gather follows the artist pass on ONE stream (a fork after it had cost
    // ~30 us of cross-stream wait on the step's critical path); the library
    // stream waits for the artist pass (its counters) before the read-back.
    // (not for a dense split: there the bucketed aggregation is the critical
    // path and the artist pass + gather beside it slowed configs[4] 16.9 ->
    // 17.2 ms/step)
    const bool art_side = c->text_deferred && spans_beside && art_ok && (MSA_ARTIST_SIDE_DENSE || !c->dense_w);
    if (art_side) {
        HIPC(c, hipStreamWaitEvent(c->side, c->ev_fix, 0));
        if ((rc = launch_artist_count(c, c->side))) return rc;
        c->artist_spec = true;
        HIPC(c, hipEventRecord(c->ev_art, c->side));
        HIPC(c, hipStreamWaitEvent(c->side, c->ev_spans, 0));
        if ((rc = launch_text(c, c->side))) return rc;
        HIPC(c, hipEventRecord(c->ev_join, c->side));
        c->side_pending = true;
    }
#else
    const bool art_side = false;
#endif
    if (!c->dense_w && (rc = build_word_lists(c))) return rc;  // (dense: the aggregation counted the entries)
#if MSA_LISTS_BEFORE_SPANS
    // the slot lists need the tables only, not the spans: they run behind
    // k_miss_agg while the spans (rank2, slowed by the token pass beside them)
    // finish; everything below waits for the spans
#if MSA_ARTIST_EARLY
    // the artist pass needs the keys only: it waits for k_rec_fix, not for the
    // offset scans behind it on rank2 (it starts as k_miss_agg's workgroups
    // leave the CUs, ~80 us earlier); the scans are waited for after it
    if (spans_beside && !art_side) HIPC(c, hipStreamWaitEvent(c->stream, c->ev_fix, 0));
#else
    if (spans_beside) HIPC(c, hipStreamWaitEvent(c->stream, c->ev_spans, 0));
#endif
#endif
    // the artist pass of msa_count (lines shortcut) right here, before the
    // read-back: it needs only the split's keys, and its counters come back
    // with the split's -- the text column's gather (launched by msa_count)
    // then no longer waits behind a second round trip and the artist kernels
    // (an exact-reader input resets the table in msa_count)
    if (art_side) {
        HIPC(c, hipStreamWaitEvent(c->stream, c->ev_art, 0));
    } else if (art_ok) {
        if ((rc = launch_artist_count(c))) return rc;
        c->artist_spec = true;
    }
#if MSA_LISTS_BEFORE_SPANS && MSA_ARTIST_EARLY
    if (spans_beside) HIPC(c, hipStreamWaitEvent(c->stream, c->ev_spans, 0));
#endif
    // text.csv's gather forked here, ahead of the read-back's copies (it needs
    // nothing the host reads back): it runs during the copies, the host's
    // header work and msa_count's launches instead of after them
    if (c->text_deferred) {
        int trc;
        if ((trc = start_text_side(c))) return trc;
    }
    HIPC(c, hipMemcpyAsync(c->pin, c->ctr.p, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
    u64 hend = c->n;
    static const u64 kHead = kPinHead;
    std::vector<unsigned char> hdr(std::min<u64>(c->n, kHead) + 1);
    if (!c->cont) {
        if (nterm > 0)
            HIPC(c, hipMemcpyAsync(c->pin + kPinSmall, c->rec_start.as<u64>() + 1, 8, hipMemcpyDeviceToHost, c->stream));
        if (c->n)
            HIPC(c, hipMemcpyAsync(c->pin + 1024, c->in, std::min<u64>(c->n, kHead), hipMemcpyDeviceToHost, c->stream));
    }
    HIPC(c, hipStreamSynchronize(c->stream));
    memcpy(&c->h_ctr, c->pin, sizeof(Counters));
    c->prev_distinct = c->h_ctr.s_claimed + c->h_ctr.m_claimed;
    c->have_hist = true;
    c->l_occ_last = c->h_ctr.l_occ;
    if (c->dense_w) {
        // a bucket past its LDS table or the planes (OVF_DENSE from the
        // device: tables from now on), or a log partition that overflowed
        // (its flush went into the HBM tables; the logs grow below): the split
        // runs again (do_split)
        if (c->h_ctr.overflow & OVF_DENSE) c->dense_veto = true;
        if (c->h_ctr.mlog_full) c->h_ctr.overflow |= OVF_DENSE | OVF_MLOG;  // (OVF_MLOG: the logs double)
    }
    // the slots this split claimed are cleared by the next one's prologue even
    // when this split fails below (a bad header) or no msa_count follows; an
    // artist table that overflowed its list is wiped whole next time (a dense
    // split claims none)
    set_used_prev(c);
    if (c->artist_spec) {
        c->a_used_prev = std::min<u64>(c->h_ctr.a_claimed, c->a_slots / 2);
        if (c->h_ctr.overflow & OVF_A) c->a_dirty = true;
    }
    c->mb_prev = c->h_ctr.k3_misses;
    if (c->h_ctr.mlog_full) {  // the logs were too small for this input's misses: 25 % more than all of
                               // them -- doubled when misses were dropped (OVF_MLOG: this split runs
                               // again) and that would not be more (a partition fuller than the rest)
        u64 want = (c->h_ctr.k3_misses + c->h_ctr.mlog_full) / 4 * 5;
        if (c->h_ctr.overflow & OVF_MLOG)
            want = std::max<u64>(want, 2 * std::max<u64>(c->mlog_want, c->mlog_cap_last * (u64)c->cus * msa_tok_wgcu() * MSA_MLOG_PARTS));
        c->mlog_want = std::max<u64>(c->mlog_want, want);
    }
    if (!c->cont) {
        if (nterm > 0) memcpy(&hend, c->pin + kPinSmall, 8);
        if (c->n) memcpy(hdr.data(), c->pin + 1024, std::min<u64>(c->n, kHead));
    }
    if (c->cont) {
        if ((rc = check_split_overflow(c, false))) return rc;
        return split_columns_rest(c, want_text, std::string(), std::string());
    }
    // header record = record 0 = [0, start of record 1), terminator included:
    // parse_csv_line strips trailing '\n' / '\r' itself (parallel_spotify.c:267-270, h_parse_header)
    if (hend > c->n) hend = c->n;
    if (hend > kHead) {  // a header longer than the bytes read with the counters
        hdr.resize(hend + 1);
        HIPC(c, hipMemcpy(hdr.data(), c->in, hend, hipMemcpyDeviceToHost));
    }
    std::string al, tl;
    if (!h_parse_header(hdr.data(), hend, al, tl)) return fail(c, MSA_ERR_BADHEADER, "Unable to parse dataset header");
    memset(c->sum.artist_label, 0, 128);
    memset(c->sum.text_label, 0, 128);
    strncpy(c->sum.artist_label, al.c_str(), 127);
    strncpy(c->sum.text_label, tl.c_str(), 127);
    h_sanitize(al, c->sum.artist_file);
    h_sanitize(tl, c->sum.text_file);

    // text.csv's header line is "<label>\n"; compute_header_length (parallel_spotify.c:444-459)
    // stops at the label's first '\n', so the rest of a multi-line label is read back as
    // lyrics by the text pass (918-941).  Tokenise that remainder too (FLAT scan).
    c->extra_len = 0;
    {
        std::string th = c->sum.text_label[0] ? c->sum.text_label : "Texts";
        const size_t nl = th.find('\n');
        if (nl != std::string::npos) {
            std::string rem = th.substr(nl + 1);
            rem.push_back('\n');
            c->extra_len = rem.size();
            HIPC(c, ensure(c->extra, c->extra_len + MSA_INPUT_PAD + MSA_CHUNK));
            HIPC(c, hipMemsetAsync(c->extra.p, 0, c->extra_len + MSA_INPUT_PAD + MSA_CHUNK, c->stream));
            HIPC(c, hipMemcpyAsync(c->extra.p, rem.data(), rem.size(), hipMemcpyHostToDevice, c->stream));
            State *d_zero = reinterpret_cast<State *>(c->small.as<char>() + 2048);
            HIPC(c, hipMemsetAsync(d_zero, 0, sizeof(State), c->stream));
            ScanArgs f = a;  // same tables and counters
            f.buf = c->extra.as<u8>();
            f.seg_begin = 0;
            f.seg_end = c->extra_len;
            f.nchunks = 1;
            f.carry = d_zero;
            f.sums = nullptr;
            f.lpos_tag = MSA_POS_EXTRA;
            if (c->dense_w) {  // the remainder's words would go into the tables: again, through the tables
                c->dense_veto = true;
                c->h_ctr.overflow |= OVF_DENSE;
                return fail(c, MSA_ERR_CAPACITY, "dense word entries and a multi-line text label: split again");
            }
            HIPC(c, msa_launch_scan(f, 2, c->stream));
            // the remainder's words may be new keys: list the tables again
            if ((rc = reset_ctr(c, &Counters::s_claimed))) return rc;
            if ((rc = reset_ctr(c, &Counters::m_claimed))) return rc;
            if ((rc = build_word_lists(c))) return rc;
            if ((rc = sync_counters(c))) return rc;
        }
    }
    std::string ah = c->sum.artist_label[0] ? c->sum.artist_label : "Artists";
    std::string th = c->sum.text_label[0] ? c->sum.text_label : "Texts";
    ah.push_back('\n');
    th.push_back('\n');
    if ((rc = check_split_overflow(c, false))) return rc;
    return split_columns_rest(c, want_text, ah, th);
}

// The split with ht_resize semantics (parallel_spotify.c:130-132): a table
// that overflows is grown and the pass repeated, so no input cardinality
// makes the call fail.
static int do_split(msa_ctx *c, int flags) {
    int rc = MSA_OK;
    for (int attempt = 0;; ++attempt) {
        ++c->split_attempts;
        rc = split_once(c, flags);
        if (rc != MSA_ERR_CAPACITY || !(c->h_ctr.overflow & kSplitOvf) || attempt == 11) return rc;
        // a table split that overflowed the S / M tables found more distinct
        // words than they hold: high cardinality, so the repeat takes the dense
        // entries (no HBM word table to grow) instead of growing the tables --
        // once; a split that is not dense-eligible grows them as before.  (A
        // cold run had first counted configs[4] through two rounds of growing
        // tables: the dense switch needs a count, and only a finished split
        // gave one.)
        if (!c->dense_w && (c->h_ctr.overflow & (OVF_S | OVF_M)) && c->dense_on && !c->dense_veto &&
            c->prev_distinct < c->dense_min) {
            c->prev_distinct = c->dense_min;
            c->h_ctr.overflow &= ~(u64)(OVF_S | OVF_M);
        }
        grow_tables(c, kSplitOvf);
        int wrc;
        if ((wrc = ensure_tables(c)) || (wrc = wipe_tables(c))) return wrc;
    }
}


// ------------------------------------------------------------------ stage 2
// Artist keying with table growth (ht_resize semantics, 130-132).
static int artist_keys(msa_ctx *c, const u8 *col, const u64 *ar_start, bool lines, u64 nrec, u64 short_base, u64 bytes) {
    int rc;
    for (int attempt = 0;; ++attempt) {
        prof_begin(c, ST_ARTIST_KEYS);
        HIPC(c, msa_launch_artist_key(col, ar_start, lines ? c->aoff.as<u64>() : nullptr,
                                      lines ? c->alen.as<u64>() : nullptr, c->a_hdr_len, nrec, c->arena.as<u8>(),
                                      c->key_off.as<u64>(), c->key_len.as<u32>(), c->key_slot.as<u64>(),
                                      c->a_tab.as<u64>(), c->a_slots - 1, c->a_list.as<u32>(), c->a_slots / 2,
                                      c->ctr.as<Counters>(), short_base, c->cus, c->ablate, c->stream));
        prof_end(c, ST_ARTIST_KEYS, bytes);
        if ((rc = sync_counters(c))) return rc;
        if (!(c->h_ctr.overflow & OVF_A) || attempt >= 12) return MSA_OK;
        grow_tables(c, OVF_A);
        if ((rc = reset_artist_table(c))) return rc;
    }
}

// Long words (> 16 bytes): table of their occurrences recorded by the scan.
static void launch_long_words(msa_ctx *c, u64 nl) {
    prof_begin(c, ST_LONG_WORDS);
    (void)msa_launch_long(c->in, c->n, c->extra.as<u8>(), c->extra_len, c->l_pos.as<u64>(), nl, c->l_len.as<u32>(),
                          c->l_slot.as<u64>(), c->l_tab.as<u64>(), c->lt_slots - 1, c->l_list.as<u32>(),
                          c->lt_slots / 2, c->ctr.as<Counters>(), c->stream);
    prof_end(c, ST_LONG_WORDS, nl * 64);
}
// A long-word pass that has to run again (the artist stage restarted and its
// counter reset dropped the pass's overflow / collision flags): its table and
// claim count start over; the flags are raised again by the new pass.
static int wipe_long_table(msa_ctx *c) {
    int rc;
    if ((rc = wipe_one(c, c->l_tab, c->lt_slots, 4, c->lt_used_prev))) return rc;
    return reset_ctr(c, &Counters::l_claimed);
}

// The artist pass of the lines shortcut (k_artist_count + merge + h2 check)
// over the split's keys, on the library stream.
static int launch_artist_count(msa_ctx *c, hipStream_t st) {
    if (!st) st = c->stream;
    const u64 nrec = c->nrec;
    // flush logs of the per-CU tables: (workgroup, 16 partitions) x cap
    // entries of 32 B; a workgroup holds <= min(6144, its records) keys
    const u64 wgs = std::max<u64>(1, std::min<u64>((nrec + 1023) / 1024, (u64)c->cus));  // k_artist_count's grid
    const u64 per_wg = (nrec + wgs - 1) / wgs;
    const u32 alog_cap = (u32)std::min<u64>(1024, std::max<u64>(64, per_wg / 8));
    HIPC(c, ensure(c->alog, (size_t)c->cus * 16 * alog_cap * 32));
    HIPC(c, ensure(c->alog_n, (size_t)c->cus * 16 * 4));
    prof_begin(c, ST_ARTIST_KEYS, st);
    HIPC(c, msa_launch_artist_count(c->alen.as<u64>(), c->key_len.as<u32>(), c->kh1.as<u64>(), c->kh2.as<u64>(), nrec,
                                    c->a_tab.as<u64>(), c->a_slots - 1, c->a_list.as<u32>(), c->a_slots / 2,
                                    c->ctr.as<Counters>(), c->cus, c->ablate, c->alog.as<ulonglong2>(),
                                    c->alog_n.as<u32>(), alog_cap, st));
    prof_end(c, ST_ARTIST_KEYS, nrec * 28, st);
    return MSA_OK;
}

static int do_count(msa_ctx *c) {
    int rc;
    if (c->stage < 1) return fail(c, MSA_ERR_ARG, "msa_count before msa_split_columns");
    if (c->stage >= 2) return MSA_OK;  // already counted: the tables are final (a second pass would add twice)
    // a label with a '\n' (its rest is read as artist records): records != lines
    bool exact = c->artist_exact || c->artist_piece_set || c->a_hdr_getline < c->a_hdr_len;
    const u64 nl = std::min<u64>(c->h_ctr.l_occ, c->l_occ_cap);  // final since the split's read-back
    {  // the long-word table from the occurrences: distinct long words <= nl,
       // so 3 slots per occurrence never overflow (growing it round by round
       // had cost a cold configs[4] run four long-word passes)
        const u32 lt_need = std::min<u32>(26, log2_ceil(nl * 3 + 1));
        if (lt_need > c->lt_log2) {
            c->lt_log2 = lt_need;
            if ((rc = ensure_tables(c))) return rc;
        }
    }
    bool long_ok = false;   // the long-word pass ran and its flags are in h_ctr
    bool long_ran = false;  // the long-word table holds a pass's counts
    if (!exact) {
        // every artist line is one artist.csv record: count the keys k_rec_spans
        // built (no record reader over artist.csv); the long-word table goes in
        // the same launch sequence, and ONE counter read-back settles both (and
        // the column lengths).  The split's a_quoted flag says whether the
        // shortcut held -- if not, start over with the exact reader.
        for (int attempt = 0;; ++attempt) {
            // the first attempt may have run already, at the end of the split
            // (its counters came back with the split's read-back)
            if (attempt > 0 || !c->artist_spec) {
                if ((rc = launch_artist_count(c))) return rc;
            }
            if (attempt == 0) {
                if ((rc = start_text_side(c))) return rc;  // text.csv beside this read-back and the ranking
                launch_long_words(c, nl);
                long_ran = true;
                HIPC(c, launch_artist_col(c, true));   // artist.csv beside text.csv and the ranking
            }
            if ((rc = sync_counters(c))) return rc;
            long_ok = attempt == 0;
            if (!(c->h_ctr.overflow & OVF_A) || attempt >= 12) break;
            grow_tables(c, OVF_A);
            if ((rc = reset_artist_table(c))) return rc;  // clears overflow + collision: the long stage reruns
        }
        if (c->h_ctr.a_quoted) {
            if (c->h_ctr.a_quoted & 2) c->a_long_cap = std::max<u64>(c->a_long_cap * 4, c->h_ctr.a_long * 2);
            exact = true;
            long_ok = false;
            if ((rc = reset_artist_table(c))) return rc;
            c->artist_spec = false;  // its counts are gone with the table
        } else {
            c->nrec_a = c->h_ctr.songs;
        }
    }
    if (exact && c->artist_spec) {
        // the split ran the lines shortcut's count, but this input takes the exact reader
        if ((rc = reset_artist_table(c))) return rc;
    }
    c->artist_spec = false;
    if (exact) {
        HIPC(c, launch_artist_col(c));  // read below; the arena it copies keys from is rewritten below
        if ((rc = resolve_col_lens(c))) return rc;
        // the artist pass over artist.csv records from its getline header end (or
        // the segment msa_segment_set chose for a shard)
        const u64 b = c->a_beg, e = c->a_end;
        State init{0, b, 0, 0, 0, 0}, fin;
        if ((rc = run_scan_fn(c, c->acol.as<u8>(), b, e, init, &fin, ST_ARTIST_SUMMARY))) return rc;
        const u64 nterm = fin.rec;
        const u64 nra = nterm + (fin.rs < e ? 1 : 0);
        const u64 cap = nterm + 2;
        HIPC(c, ensure(c->ar_start, cap * 8));
        // arena: keys rewritten by duplicate_field at their artist.csv offsets, then
        // one aligned 32-byte slot per record for keys built in registers
        const u64 short_base = (e + 64 + 255) & ~255ull;
        HIPC(c, ensure(c->arena, short_base + 32 * cap + 64));
        HIPC(c, ensure(c->key_off, cap * 8));
        HIPC(c, ensure(c->key_len, cap * 4));
        HIPC(c, ensure(c->key_slot, cap * 8));
        HIPC(c, hipMemcpyAsync(c->ar_start.p, &b, 8, hipMemcpyHostToDevice, c->stream));
        if (e > b) {
            ScanArgs a{};
            a.buf = c->acol.as<u8>();
            a.seg_begin = b;
            a.seg_end = e;
            a.nchunks = (u32)((e - b + MSA_CHUNK - 1) / MSA_CHUNK);
            a.carry = c->carry.as<State>();
            a.rec_start = c->ar_start.as<u64>();
            a.rec_cap = cap;
            a.ctr = c->ctr.as<Counters>();
            prof_begin(c, ST_ARTIST_SCAN);
            HIPC(c, msa_launch_scan(a, 1, c->stream));
            prof_end(c, ST_ARTIST_SCAN, (e - b) + nra * 16);
        }
        if (fin.rs < e) HIPC(c, hipMemcpyAsync(c->ar_start.as<u64>() + nra, &e, 8, hipMemcpyHostToDevice, c->stream));
        c->nrec_a = nra;
        if ((rc = artist_keys(c, c->acol.as<u8>(), c->ar_start.as<u64>(), false, nra, short_base, (e - b) * 2 + nra * 48)))
            return rc;
    }
    // words longer than 16 bytes (their table grows the same way)
    for (int attempt = 0;; ++attempt) {
        if (!long_ok) {
            if (long_ran && attempt == 0 && (rc = wipe_long_table(c))) return rc;
            launch_long_words(c, nl);
            long_ran = true;
            if ((rc = sync_counters(c))) return rc;
        }
        long_ok = false;
        if (!(c->h_ctr.overflow & OVF_LT) || attempt >= 12) break;
        // the artist stage is done: only the long-word table and its counters restart
        const u64 keep_collision = c->h_ctr.collision;
        grow_tables(c, OVF_LT);
        if ((rc = ensure_tables(c))) return rc;
        if ((rc = wipe_one(c, c->l_tab, c->lt_slots, 4, c->lt_used_prev))) return rc;
        if ((rc = reset_ctr(c, &Counters::l_claimed))) return rc;
        if ((rc = reset_ctr(c, &Counters::overflow))) return rc;
        if (!keep_collision && (rc = reset_ctr(c, &Counters::collision))) return rc;
    }
    set_used_prev(c);
    c->lt_used_prev = std::min<u64>(c->h_ctr.l_claimed, c->lt_slots / 2);
    c->a_used_prev = std::min<u64>(c->h_ctr.a_claimed, c->a_slots / 2);
    if (c->h_ctr.overflow) return fail(c, MSA_ERR_CAPACITY, "table capacity overflow (flags 0x%llx)",
                                       (unsigned long long)c->h_ctr.overflow);
    if (c->h_ctr.collision)
        return fail(c, MSA_ERR_COLLISION, "64-bit key hash collision detected (%llu occurrences)",
                    (unsigned long long)c->h_ctr.collision);
    c->sum.total_songs = (long long)c->nrec_a;
    c->sum.total_words = (long long)c->h_ctr.total_words;
    c->sum.n_words = c->h_ctr.s_claimed + c->h_ctr.m_claimed + c->h_ctr.l_claimed;
    c->sum.n_artists = c->h_ctr.a_claimed;
    c->sum.n_records = c->nrec;
    c->stage = 2;
    return MSA_OK;
}

// ------------------------------------------------------------------ stage 3
static const u64 kRadixMin = 1ull << 18;

// Order of entries equal in (count, first 16 key bytes), radix path: round r
// re-sorts the tied entries by (their run, key bytes [16 r, 16 r + 16)) with
// the radix sort, until no two adjacent keys are equal (keys are distinct).
// covered: key bytes the main sort ordered by (16, or 8 when it left K0 out:
// the first round then also orders runs equal in count and first 8 bytes; 6
// or 7 after the composite key's sort, whose sorted keys -- the set's K2
// plane -- mark the first round's runs)
static int refine_ties(msa_ctx *c, Ranked &R, int cur, const u8 *wbuf, const u8 *wextra, const u8 *arena,
                       const u64 *key_off, const u32 *key_len, u32 covered, RefineBufs &rb, hipStream_t st,
                       bool comp = false) {
    const u64 n = R.n;
    HIPC(c, hipMemcpyAsync(R.order.p, R.V[cur].p, n * 4, hipMemcpyDeviceToDevice, st));
    // per block of entries: head / tie counts (t_head / t_tie) and their scans (t_runid / t_tpos)
    const u64 nb0 = msa_tie_blocks(n);
    for (DevBuf *b : {&rb.t_head, &rb.t_tie, &rb.t_runid, &rb.t_tpos}) HIPC(c, ensure(*b, nb0 * 8));
    const u64 nbb = (nb0 + 1023) / 1024 + 1;
    HIPC(c, ensure(rb.t_bsum, 2 * nbb * 8));
    HIPC(c, ensure(rb.t_total, 64));
    const u64 *K2 = R.K[cur][0].as<u64>(), *K1 = comp ? K2 : R.K[cur][1].as<u64>();
    const u64 *K0 = covered == 16 ? R.K[cur][2].as<u64>() : nullptr;
    const u32 *Vc = R.V[cur].as<u32>();
    const u64 *Pc = nullptr;
    u64 mc = n;
    for (u32 r = 1; r < 4096; ++r) {
        const u64 nb = msa_tie_blocks(mc);
        // t_total: [0] runs, [1] tied entries, [2] a run longer than TIE_SEG (k_tie_count)
        HIPC(c, hipMemsetAsync(rb.t_total.as<u64>() + 2, 0, 8, st));
        HIPC(c, msa_launch_tie_count(K2, K1, K0, mc, rb.t_head.as<u64>(), rb.t_tie.as<u64>(),
                                     rb.t_total.as<u64>() + 2, st));
        HIPC(c, msa_exclusive_scan2(rb.t_head.as<u64>(), nb, rb.t_runid.as<u64>(), rb.t_bsum.as<u64>(),
                                    rb.t_total.as<u64>(), rb.t_tie.as<u64>(), nb, rb.t_tpos.as<u64>(),
                                    rb.t_bsum.as<u64>() + nbb, rb.t_total.as<u64>() + 1, st));
        u64 mb[2] = {0, 0};
        HIPC(c, hipMemcpyAsync(mb, rb.t_total.as<u64>() + 1, 16, hipMemcpyDeviceToHost, st));
        HIPC(c, hipStreamSynchronize(st));
        const u64 m = mb[0];
        const bool seg = c->tie_seg && !mb[1];  // every run short: k_tie_seg orders them
        if (c->ablate & 4096) fprintf(stderr, "refine_ties: n %llu round %u ties %llu\n", (unsigned long long)n, r,
                                      (unsigned long long)m);
        if (!m) return MSA_OK;
        for (int s = 0; s < 3; ++s) {
            for (int k = 0; k < 3; ++k) HIPC(c, ensure(rb.t_K[s][k], m * 8));
            HIPC(c, ensure(rb.t_V[s], m * 4));
        }
        HIPC(c, ensure(rb.t_Vn, m * 4));
        HIPC(c, ensure(rb.t_Pn, m * 8));
        HIPC(c, ensure(rb.t_Vc, m * 4));
        HIPC(c, ensure(rb.t_Pc, m * 8));
        u64 *k2[3], *k1[3], *k0[3];
        u32 *vv[3];
        for (int s = 0; s < 3; ++s) {
            k2[s] = rb.t_K[s][0].as<u64>();
            k1[s] = rb.t_K[s][1].as<u64>();
            k0[s] = rb.t_K[s][2].as<u64>();
            vv[s] = rb.t_V[s].as<u32>();
        }
        HIPC(c, msa_launch_tie_build(K2, K1, K0, mc, rb.t_runid.as<u64>(), rb.t_tpos.as<u64>(), Vc, Pc,
                                     covered + 16 * (r - 1), R.K[0][1].as<u64>(), R.K[0][2].as<u64>(), R.ref.as<u64>(), wbuf, wextra, c->l_pos.as<u64>(), c->l_len.as<u32>(), arena,
                                     key_off, key_len, k2[0], k1[0], k0[0], vv[0], rb.t_Vn.as<u32>(),
                                     rb.t_Pn.as<u64>(), st));
        int o = 1;
        if (seg) HIPC(c, msa_launch_tie_seg(k2[0], k1[0], k0[0], vv[0], m, k2[1], k1[1], k0[1], vv[1], st));
        else HIPC(c, msa_radix_sort(k2, k1, k0, vv, m, &o, rb.sort_scratch.as<u8>(), st));
        HIPC(c, msa_launch_tie_apply(vv[o], rb.t_Vn.as<u32>(), rb.t_Pn.as<u64>(), m, R.order.as<u32>(),
                                     rb.t_Vc.as<u32>(), rb.t_Pc.as<u64>(), R.K[0][1].as<u64>(), R.K[0][2].as<u64>(),
                                     covered < 8 ? R.K[cur][1].as<u64>() : nullptr,
                                     covered == 16 ? nullptr : R.K[cur][2].as<u64>(), st));
        K2 = k2[o];
        K1 = k1[o];
        K0 = k0[o];
        Vc = rb.t_Vc.as<u32>();
        Pc = rb.t_Pc.as<u64>();
        mc = m;
    }
    return fail(c, MSA_ERR_COLLISION, "tie refinement did not converge (equal keys in the %s table: %llu of %llu entries tied)",
                &R == &c->rw ? "word" : "artist", (unsigned long long)mc, (unsigned long long)n);
}

static bool small_sort(const msa_ctx *c, u64 n) { return c->sort_mode == 1 || (c->sort_mode == 0 && n < kRadixMin); }

// Sort + key blob of one table on stream st (the radix path -- large tables --
// reads back tie counts and runs on the library stream only).
static int sort_and_blob(msa_ctx *c, Ranked &R, const u8 *wbuf, const u8 *wextra, const u8 *arena, const u64 *key_off,
                         const u32 *key_len, int slot, u64 est, hipStream_t st, RefineBufs &rb) {
    const u64 n = R.n;
    R.host_valid = false;
    R.blob_pending = n != 0;
    if (n == 0) {
        R.blob_len = 0;
        return MSA_OK;
    }
    for (int s = 1; s < 3; ++s) {
        for (int k = 0; k < 3; ++k) HIPC(c, ensure(R.K[s][k], n * 8));
        HIPC(c, ensure(R.V[s], n * 4));
    }
    u64 *k2[3], *k1[3], *k0[3];
    u32 *vv[3];
    for (int s = 0; s < 3; ++s) {
        k2[s] = R.K[s][0].as<u64>();
        k1[s] = R.K[s][1].as<u64>();
        k0[s] = R.K[s][2].as<u64>();
        vv[s] = R.V[s].as<u32>();
    }
    int cur = 1;
    // large tables: LSD radix sort (msa_sort.hip); small ones: LDS bitonic
    // tiles, then one ranking launch (<= 64 Ki keys) or merge passes
    // (launch-bound sizes).  MSA_SORT=radix|merge forces one.
    HIPC(c, ensure(R.order, n * 4));
    HIPC(c, ensure(R.len, n * 8));
    HIPC(c, ensure(R.off, (n + 1) * 8));
    HIPC(c, ensure(c->blob_tot, 64));
    HIPC(c, ensure(R.scan_bsum, ((n + 1023) / 1024 + 1) * 8));
    // the blob length stays on the device until do_rank's one sync (the scan
    // leaves it in blob_tot[slot]): the blob is sized from what the host knows
    // (the last run's length, or an estimate) and k_blob_write skips keys past
    // that capacity (do_rank redoes them)
    bool lens_done = false;
    if (small_sort(c, n) && n <= msa_rank_small_max()) {
        // up to 64 Ki keys: tile sort + two ranking launches + the offsets' scan
        HIPC(c, ensure(R.rank_cnt, msa_rank_small_scratch(n)));
        HIPC(c, msa_launch_rank_small(k2, k1, k0, vv, n, R.ref.as<u64>(), wbuf, wextra, c->l_pos.as<u64>(),
                                      c->l_len.as<u32>(), arena, key_off, key_len, R.order.as<u32>(),
                                      R.len.as<u64>(), R.off.as<u64>(), R.scan_bsum.as<u64>(),
                                      c->blob_tot.as<u64>() + slot, R.rank_cnt.as<u32>(), st));
        lens_done = true;
    } else if (!small_sort(c, n)) {
        HIPC(c, ensure(rb.sort_scratch, msa_radix_scratch_bytes(n)));
        // words: the passes over K0 (key bytes 8..15) are left to the tie
        // refinement -- equal (count, first 8 bytes) runs are rare in a word
        // table, so a round over them is cheaper than 8 passes over all entries
        // (artists: prefixes shared by many names; MSA_SORT_K0=1 sorts K0 for words too)
        // words: the radix passes cover the first 8 key bytes (K2 / K1), the
        // tie refinement the rest; artists (long shared name prefixes) keep
        // the K0 passes too
        const bool sk0 = slot != 0;
        // words: the composite key (dense count rank + first key bytes, one
        // word; msa_sort.hip) when the counts take few enough distinct values
        u32 gB = ~0u;
        if (!sk0 && c->comp_sort && R.vary_ok) {
            HIPC(c, ensure(R.comp, n * 8));
            HIPC(c, ensure(R.cset, msa_comp_scratch_bytes()));
            u64 *wsk = nullptr;
            u32 *vk = nullptr;
            HIPC(c, msa_radix_sort_comp(k2, k1, k0, vv, n, &cur, rb.sort_scratch.as<u8>(), st, R.vary.as<u64>(),
                                        R.comp.as<u64>(), R.cset.as<u8>(), &gB, &wsk, &vk));
            if (vk) {  // the sorted values stayed in the last pass's buffer (set 1 or 2): set cur's V
                if (R.V[1].p == vk) std::swap(R.V[cur], R.V[1]);
                else if (R.V[2].p == vk) std::swap(R.V[cur], R.V[2]);
                else return fail(c, MSA_ERR_HIP, "radix sort: sorted values in an unknown buffer");
            }
            if (wsk) {  // the sorted keys stayed in a pass buffer (a K0 plane of sets 1/2): it becomes set cur's K2
                bool swapped = false;
                for (int s2 = 1; s2 < 3 && !swapped; ++s2)
                    if (R.K[s2][2].p == wsk) {
                        std::swap(R.K[cur][0], R.K[s2][2]);
                        swapped = true;
                    }
                if (!swapped) return fail(c, MSA_ERR_HIP, "radix sort: sorted keys in an unknown buffer");
            }
        }
        int rc;
        if (gB != ~0u) {
            if ((rc = refine_ties(c, R, cur, wbuf, wextra, arena, key_off, key_len, 8 - gB, rb, st, true))) return rc;
            HIPC(c, msa_comp_finish(R.K[cur][0].as<u64>(), n, R.cset.as<u8>(), gB, st));
        } else {
            HIPC(c, msa_radix_sort(k2, k1, k0, vv, n, &cur, rb.sort_scratch.as<u8>(), st,
                                   R.vary_ok ? R.vary.as<u64>() : nullptr, sk0));
            if ((rc = refine_ties(c, R, cur, wbuf, wextra, arena, key_off, key_len, sk0 ? 16 : 8, rb, st))) return rc;
        }
    } else {
        HIPC(c, msa_launch_sort(k2, k1, k0, vv, n, &cur, st));
        HIPC(c, msa_launch_fixup(R.K[cur][0].as<u64>(), R.K[cur][1].as<u64>(), R.K[cur][2].as<u64>(),
                                 R.V[cur].as<u32>(), n, R.ref.as<u64>(), wbuf, wextra, c->l_pos.as<u64>(),
                                 c->l_len.as<u32>(), arena, key_off, key_len, R.order.as<u32>(), st));
    }
    // key blob in rank order
    HIPC(c, ensure(R.counts, n * 8));
    HIPC(c, ensure(R.scan_total, 64));
    HIPC(c, ensure(R.scan_bsum, ((n + 1023) / 1024 + 1) * 8));
    // after a full sort, rank i's key planes are R.K[cur][*][i] (read in order)
    const u64 *ks2 = lens_done ? nullptr : R.K[cur][0].as<u64>();
    const u64 *ks1 = lens_done ? nullptr : R.K[cur][1].as<u64>();
    const u64 *ks0 = lens_done ? nullptr : R.K[cur][2].as<u64>();
    if (!lens_done)
        HIPC(c, msa_launch_blob(R.order.as<u32>(), n, R.ref.as<u64>(), R.K[0][1].as<u64>(), R.K[0][2].as<u64>(),
                                R.cnt.as<u64>(), wbuf, wextra, c->l_pos.as<u64>(), c->l_len.as<u32>(), arena, key_off,
                                key_len, R.len.as<u64>(), R.off.as<u64>(), R.scan_bsum.as<u64>(),
                                c->blob_tot.as<u64>() + slot, nullptr, nullptr, 0, st, 0, ks2, ks1, ks0, R.lthr));
    HIPC(c, ensure(R.blob, std::max<u64>(est, R.blob_len) + 16));
    R.blob_cap = R.blob.cap - 16;
    HIPC(c, msa_launch_blob(R.order.as<u32>(), n, R.ref.as<u64>(), R.K[0][1].as<u64>(), R.K[0][2].as<u64>(),
                            R.cnt.as<u64>(), wbuf, wextra, c->l_pos.as<u64>(), c->l_len.as<u32>(), arena, key_off, key_len,
                            R.len.as<u64>(), R.off.as<u64>(), R.scan_bsum.as<u64>(), R.scan_total.as<u64>(),
                            R.blob.as<u8>(), R.counts.as<u64>(), R.blob_cap, st, 1, ks2, ks1, ks0, R.lthr));
    R.pending = BlobArgs{wbuf, wextra, arena, key_off, key_len, ks2, ks1, ks0, R.lthr};
    return MSA_OK;
}

static hipError_t grow_keep(DevBuf &b, size_t bytes, size_t keep, hipStream_t s);

// tables: bit 0 words, bit 1 artists (a table left out keeps its ranking)
static int do_rank(msa_ctx *c, int tables = 3) {
    int rc;
    if (c->stage < 2) return fail(c, MSA_ERR_ARG, "msa_rank before msa_count");
    // a table merged by msa_import_ranked is ranked already (its count tables
    // are not the merged table: ranking them again would write entries for keys
    // the ranked arrays were not sized for)
    tables &= ~c->ranked_only;
    if (!tables) return MSA_OK;
    if ((rc = start_text_side(c))) return rc;
    // words
    Ranked &W = c->rw;
    const bool dw = (tables & 1) != 0, da = (tables & 2) != 0;
    if (dw) {
        W.n = c->sum.n_words;
        W.lthr = c->h_ctr.s_claimed + c->h_ctr.m_claimed;
    }
    prof_begin(c, ST_RANK_WORDS);
    // dense split: entries [0, lthr) are written already (k_mb_agg<true>), the
    // long words' are appended; the planes were sized for them by the split
    const bool dense = dw && c->dense_w && !c->merged_w;
    if (dense && W.n) {
        // the split sized the planes for the long words its long-word table
        // could hold then; msa_count may have grown that table since (OVF_LT):
        // the planes grow too, keeping the dense entries [0, lthr)
        const u64 nd = W.lthr;
        for (int k = 0; k < 3; ++k) HIPC(c, grow_keep(W.K[0][k], W.n * 8, nd * 8, c->stream));
        HIPC(c, grow_keep(W.V[0], W.n * 4, nd * 4, c->stream));
        HIPC(c, grow_keep(W.ref, W.n * 8, nd * 8, c->stream));
        HIPC(c, grow_keep(W.cnt, W.n * 8, nd * 8, c->stream));
    }
    if (dense && W.n) {
        EntryArgs ea{};
        const u64 nd = W.lthr;
        ea.l_tab = c->l_tab.as<u64>();
        ea.l_list = c->l_list.as<u32>();
        ea.nl = c->h_ctr.l_claimed;
        ea.buf = c->in;
        ea.extra = c->extra.as<u8>();
        ea.l_pos = c->l_pos.as<u64>();
        ea.l_len = c->l_len.as<u32>();
        ea.K2 = W.K[0][0].as<u64>() + nd;
        ea.K1 = W.K[0][1].as<u64>() + nd;
        ea.K0 = W.K[0][2].as<u64>() + nd;
        ea.val = W.V[0].as<u32>() + nd;
        ea.ref = W.ref.as<u64>() + nd;
        ea.cnt = W.cnt.as<u64>() + nd;  // the dense entries wrote theirs (the small-table ranking reads it)
        ea.vbase = nd;
        W.vary_ok = !small_sort(c, W.n);
        ea.vary = W.vary_ok ? W.vary.as<u64>() : nullptr;  // the dense planes' OR / AND are there already
        HIPC(c, msa_launch_word_entries(ea, c->stream));
    } else if (dw && W.n) {
        for (int k = 0; k < 3; ++k) HIPC(c, ensure(W.K[0][k], W.n * 8));
        HIPC(c, ensure(W.V[0], W.n * 4));
        HIPC(c, ensure(W.ref, W.n * 8));
        HIPC(c, ensure(W.cnt, W.n * 8));
        EntryArgs ea{};
        ea.s_tab = c->s_tab.as<u64>();
        ea.s_list = c->s_list.as<u32>();
        ea.ns = c->h_ctr.s_claimed;
        ea.m_tab = c->m_tab.as<u64>();
        ea.m_list = c->m_list.as<u32>();
        ea.nm = c->h_ctr.m_claimed;
        ea.l_tab = c->l_tab.as<u64>();
        ea.l_list = c->l_list.as<u32>();
        ea.nl = c->h_ctr.l_claimed;
        ea.buf = c->merged_w ? c->imp_w.as<u8>() : c->in;
        ea.extra = c->merged_w ? c->imp_w.as<u8>() : c->extra.as<u8>();
        ea.l_pos = c->l_pos.as<u64>();
        ea.l_len = c->l_len.as<u32>();
        ea.K2 = W.K[0][0].as<u64>();
        ea.K1 = W.K[0][1].as<u64>();
        ea.K0 = W.K[0][2].as<u64>();
        ea.val = W.V[0].as<u32>();
        ea.ref = W.ref.as<u64>();
        W.vary_ok = !small_sort(c, W.n);  // the radix sort's varying bytes, reduced while the entries are written
        // the count plane: read only by the small-table ranking's key blob (the
        // radix path's blob reads the sorted ~count plane)
        ea.cnt = W.vary_ok ? nullptr : W.cnt.as<u64>();
        if (W.vary_ok) {
            HIPC(c, ensure(W.vary, 64));
            HIPC(c, hipMemsetAsync(W.vary.p, 0, 24, c->stream));
            HIPC(c, hipMemsetAsync(W.vary.as<u64>() + 3, 0xFF, 24, c->stream));
            ea.vary = W.vary.as<u64>();
        }
        HIPC(c, msa_launch_word_entries(ea, c->stream));
    }
    const u8 *wbuf = c->merged_w ? c->imp_w.as<u8>() : c->in;
    const u8 *wextra = c->merged_w ? c->imp_w.as<u8>() : c->extra.as<u8>();
    const u64 west = c->h_ctr.s_claimed * 8 + c->h_ctr.m_claimed * 16 + c->h_ctr.l_claimed * 48;
    // artists: on their own stream beside the words when both tables take the
    // small-table sort (a chain of short latency-bound launches each); a
    // radix-sorted artist table (configs[4]: millions of artists, its tie
    // refinement reading counts back round after round) is ranked on a host
    // thread of its own, with its own scratch, beside the words'
    Ranked &A = c->ra;
    if (da) A.n = c->sum.n_artists;
    const bool conc_small = dw && da && small_sort(c, W.n) && small_sort(c, A.n) && A.n;
    const bool conc_thread = dw && da && W.n && A.n && !small_sort(c, A.n);
    const bool conc = conc_small || conc_thread;
    hipStream_t ast = conc ? c->rank2 : c->stream;
    if (conc) {
        HIPC(c, hipEventRecord(c->ev_r2_fork, c->stream));
        HIPC(c, hipStreamWaitEvent(c->rank2, c->ev_r2_fork, 0));
    }
    // every exit after the fork joins rank2 back into the library stream (an
    // error return too: later work there must stay ordered after the artist
    // kernels still running on rank2)
    struct R2Join {
        msa_ctx *c;
        bool on;
        ~R2Join() {
            if (!on) return;
            (void)hipEventRecord(c->ev_r2_join, c->rank2);
            (void)hipStreamWaitEvent(c->stream, c->ev_r2_join, 0);
        }
    } r2_join{c, conc};
    const u8 *aarena = c->merged_a ? c->imp_a.as<u8>() : c->arena.as<u8>();
    auto rank_artists = [&]() -> int {
        int arc;
        prof_begin(c, ST_RANK_ARTISTS, ast);
        if (da && A.n) {
            for (int k = 0; k < 3; ++k) HIPC(c, ensure(A.K[0][k], A.n * 8));
            HIPC(c, ensure(A.V[0], A.n * 4));
            HIPC(c, ensure(A.ref, A.n * 8));
            HIPC(c, ensure(A.cnt, A.n * 8));
            HIPC(c, msa_launch_artist_entries(c->a_tab.as<u64>(), c->a_list.as<u32>(), A.n, aarena,
                                              c->key_off.as<u64>(), c->key_len.as<u32>(), A.K[0][0].as<u64>(),
                                              A.K[0][1].as<u64>(), A.K[0][2].as<u64>(), A.V[0].as<u32>(),
                                              A.ref.as<u64>(), A.cnt.as<u64>(), ast));
        }
        if (da && (arc = sort_and_blob(c, A, wbuf, wextra, aarena, c->key_off.as<u64>(), c->key_len.as<u32>(), 1,
                                       A.n * 32, ast, conc_thread ? c->rb[1] : c->rb[0])))
            return arc;
        prof_end(c, ST_RANK_ARTISTS, A.n * 64 + A.blob_len, ast);
        return MSA_OK;
    };
    int arc = MSA_OK;
    HIPC(c, ensure(c->blob_tot, 64));  // shared by both tables' blob scans: allocated before the thread
    if (conc_thread) {
        // the artists' entry arrays sized here, not on the ranking thread: a
        // regrowth frees a buffer, and hipFree waits for the whole device (the
        // words' passes included).  The sort's own buffers still grow there on
        // a larger table than any before -- the first runs, not steady state.
        for (int k = 0; k < 3; ++k) HIPC(c, ensure(A.K[0][k], A.n * 8));
        HIPC(c, ensure(A.V[0], A.n * 4));
        HIPC(c, ensure(A.ref, A.n * 8));
        HIPC(c, ensure(A.cnt, A.n * 8));
    }
    std::thread ath;
    struct TJoin {
        std::thread &t;
        ~TJoin() {
            if (t.joinable()) t.join();
        }
    } ath_join{ath};  // joined before r2_join records (declared after it)
    if (conc_thread)
        ath = std::thread([&] {
            if (hipSetDevice(c->device) != hipSuccess) {
                arc = fail(c, MSA_ERR_HIP, "hipSetDevice on the ranking thread");
                return;
            }
            arc = rank_artists();
        });
    if (dw && (rc = sort_and_blob(c, W, wbuf, wextra, nullptr, nullptr, nullptr, 0, west, c->stream, c->rb[0])))
        return rc;
    prof_end(c, ST_RANK_WORDS, W.n * 64 + W.blob_len);
    if (conc_thread) {
        ath.join();
        if (arc) return arc;
    } else if ((rc = rank_artists())) {
        return rc;
    }
    if (conc) {
        r2_join.on = false;
        HIPC(c, hipEventRecord(c->ev_r2_join, c->rank2));
        HIPC(c, hipStreamWaitEvent(c->stream, c->ev_r2_join, 0));
    }
    // the one read-back of the ranking: both blob lengths; a blob that did not
    // fit the capacity it was written with is grown and written again
    u64 tot[2] = {0, 0};
    if (W.blob_pending || A.blob_pending)
        HIPC(c, hipMemcpyAsync(c->pin + kPinSmall, c->blob_tot.p, sizeof tot, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    if (W.blob_pending || A.blob_pending) memcpy(tot, c->pin + kPinSmall, sizeof tot);
    bool again = false;
    for (int t = 0; t < 2; ++t) {
        Ranked &R = t ? A : W;
        if (!R.blob_pending) continue;
        R.blob_pending = false;
        R.blob_len = tot[t];
        if (R.blob_len <= R.blob_cap) continue;
        HIPC(c, ensure(R.blob, R.blob_len + 16));
        R.blob_cap = R.blob.cap - 16;
        const BlobArgs &b = R.pending;
        HIPC(c, msa_launch_blob(R.order.as<u32>(), R.n, R.ref.as<u64>(), R.K[0][1].as<u64>(), R.K[0][2].as<u64>(),
                                R.cnt.as<u64>(), b.wbuf, b.wextra, c->l_pos.as<u64>(), c->l_len.as<u32>(), b.arena,
                                b.key_off, b.key_len, R.len.as<u64>(), R.off.as<u64>(), R.scan_bsum.as<u64>(),
                                R.scan_total.as<u64>(), R.blob.as<u8>(), R.counts.as<u64>(), R.blob_cap, c->stream,
                                1, b.ks2, b.ks1, b.ks0, b.lthr));
        again = true;
    }
    if (again) HIPC(c, hipStreamSynchronize(c->stream));
    c->stage = 3;
    return MSA_OK;
}

static int fetch_ranked(msa_ctx *c, Ranked &R) {
    if (R.host_valid) return MSA_OK;
    R.h_counts.resize(R.n);
    R.h_off.resize(R.n + 1);
    R.h_blob.resize(R.blob_len + 1);
    if (R.n) {
        HIPC(c, hipMemcpy(R.h_counts.data(), R.counts.p, R.n * 8, hipMemcpyDeviceToHost));
        HIPC(c, hipMemcpy(R.h_off.data(), R.off.p, R.n * 8, hipMemcpyDeviceToHost));
        if (R.blob_len) HIPC(c, hipMemcpy(R.h_blob.data(), R.blob.p, R.blob_len, hipMemcpyDeviceToHost));
    }
    R.h_off[R.n] = R.blob_len;
    R.host_valid = true;
    return MSA_OK;
}

// ===================================================================== C ABI
extern "C" {

int msa_create(int device, msa_ctx **out) {
    if (!out) return MSA_ERR_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return MSA_ERR_HIP;
    if (device < 0 || device >= ndev) return MSA_ERR_ARG;
    if (hipSetDevice(device) != hipSuccess) return MSA_ERR_HIP;
    msa_ctx *c = new msa_ctx();
    c->device = device;
#ifdef MSA_DIAG
    if (const char *ab = getenv("MSA_ABLATE")) c->ablate = atoi(ab);
#endif
    if (const char *cs = getenv("MSA_COMP_SORT")) c->comp_sort = atoi(cs) != 0;
    if (const char *ch = getenv("MSA_CSV_HOST_MAX")) c->csv_host_max = strtoull(ch, nullptr, 10);
    if (const char *ts = getenv("MSA_TIE_SEG")) c->tie_seg = atoi(ts) != 0;
    if (const char *fo = getenv("MSA_FOLD")) c->fold = atoi(fo) != 0;
    if (const char *mb = getenv("MSA_MISS_BUCKETS")) c->mb_mode = atoi(mb);
    if (const char *mm = getenv("MSA_MISS_BUCKETS_MIN")) c->mb_min = strtoull(mm, nullptr, 10);
    if (const char *de = getenv("MSA_DENSE")) c->dense_on = atoi(de) != 0;
    if (const char *dm = getenv("MSA_DENSE_MIN")) c->dense_min = strtoull(dm, nullptr, 10);
    if (const char *me = getenv("MSA_MLOG_ENTRIES")) c->mlog_test = strtoull(me, nullptr, 10);
    if (const char *so = getenv("MSA_SORT")) c->sort_mode = !strcmp(so, "merge") ? 1 : (!strcmp(so, "radix") ? 2 : 0);
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
            c->cus = prop.multiProcessorCount;
    }
    // (round 3 measured and removed: the side stream masked off every 8th /
    // 16th CU with hipExtStreamCreateWithCUMask -- no gain)
    // text.csv's side stream at the highest priority: its gather is the step's
    // tail and the ranking beside it has slack (2.88-2.91 vs 2.92-2.96 ms/step,
    // profiles/r04_t48_ab_side_priority.txt)
    int least = 0, greatest = 0;
    (void)hipDeviceGetStreamPriorityRange(&least, &greatest);
    const hipError_t side_e = hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, greatest);
#ifndef MSA_R2_PRIO
#define MSA_R2_PRIO 0  // 1: rank2 (the spans beside the token pass, the artists' ranking) at the highest priority
#endif
    const hipError_t r2_e = MSA_R2_PRIO ? hipStreamCreateWithPriority(&c->rank2, hipStreamNonBlocking, greatest)
                                        : hipStreamCreateWithFlags(&c->rank2, hipStreamNonBlocking);
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess || side_e != hipSuccess ||
        r2_e != hipSuccess ||
        hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_aux_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_aux_join, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_r2_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_r2_join, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_scan_a, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_spans, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_fix, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_art, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_fin, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess ||
        hipHostMalloc((void **)&c->pin, kPinBytes, hipHostMallocDefault) != hipSuccess) {
        delete c;
        return MSA_ERR_HIP;
    }
    *out = c;
    return MSA_OK;
}

void msa_destroy(msa_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    c->artist_deferred = c->text_deferred = false;  // nothing reads them any more
    (void)join_side(c);
    (void)hipStreamSynchronize(c->stream);
    DevBuf *all[] = {&c->in_own, &c->sums, &c->carry, &c->btot, &c->bstate, &c->small, &c->rec_start, &c->extra, &c->exp_buf, &c->exp_meta, &c->imp_w, &c->imp_a, &c->imp_meta,
                     &c->nulrel, &c->f0, &c->tss, &c->tse, &c->span_fix, &c->alog, &c->alog_n, &c->acol, &c->alen, &c->aoff, &c->asrc, &c->apairs, &c->tcol, &c->tlen, &c->toff, &c->tsrc, &c->tpairs,
                     &c->tscan_bsum, &c->scan_bsum, &c->scan_total, &c->ar_start, &c->arena, &c->key_off,
                     &c->key_len, &c->key_slot, &c->s_tab, &c->s_list, &c->m_tab, &c->m_list, &c->l_pos, &c->l_len,
                     &c->l_slot, &c->l_tab, &c->l_list, &c->a_tab, &c->a_list, &c->ctr, &c->kh1, &c->kh2, &c->mlog, &c->mlog_n, &c->lmask, &c->blob_tot, &c->fold_buf,
                     &c->mb_hist, &c->mb_off, &c->mb_bsum, &c->mb_tot, &c->mb_out, &c->csv_len, &c->csv_pos, &c->csv_bsum, &c->csv_out};
    for (DevBuf *b : all) release(*b);
    for (Ranked *R : {&c->rw, &c->ra}) {
        for (auto &s : R->K)
            for (auto &k : s) release(k);
        for (auto &v : R->V) release(v);
        DevBuf *rb[] = {&R->ref, &R->cnt, &R->order, &R->len, &R->off, &R->blob, &R->counts, &R->scan_bsum,
                        &R->scan_total, &R->rank_cnt, &R->vary};
        for (DevBuf *b : rb) release(*b);
    }
    for (RefineBufs &rb : c->rb) {
        for (DevBuf *b : {&rb.sort_scratch, &rb.t_head, &rb.t_tie, &rb.t_runid, &rb.t_tpos, &rb.t_bsum, &rb.t_total,
                          &rb.t_Vn, &rb.t_Pn, &rb.t_Vc, &rb.t_Pc})
            release(*b);
        for (auto &s : rb.t_K)
            for (auto &k : s) release(k);
        for (auto &v : rb.t_V) release(v);
    }
    for (ProfStage &s : c->ps) {
        if (s.a) (void)hipEventDestroy(s.a);
        if (s.b) (void)hipEventDestroy(s.b);
    }
    (void)hipHostFree(c->pin);
    if (c->csv_pin) (void)hipHostFree(c->csv_pin);
    (void)hipEventDestroy(c->ev_fork);
    (void)hipEventDestroy(c->ev_join);
    (void)hipEventDestroy(c->ev_r2_fork);
    (void)hipEventDestroy(c->ev_fin);
    (void)hipEventDestroy(c->ev_r2_join);
    (void)hipEventDestroy(c->ev_scan_a);
    (void)hipEventDestroy(c->ev_spans);
    (void)hipEventDestroy(c->ev_fix);
    (void)hipEventDestroy(c->ev_art);
    (void)hipStreamDestroy(c->side);
    (void)hipStreamDestroy(c->rank2);
    (void)hipStreamDestroy(c->aux);
    (void)hipEventDestroy(c->ev_aux_fork);
    (void)hipEventDestroy(c->ev_aux_join);
    (void)hipStreamDestroy(c->stream);
    delete c;
}

const char *msa_last_error(const msa_ctx *c) { return c ? c->err.c_str() : "no context"; }
void *msa_stream(msa_ctx *c) { return c ? (void *)c->stream : nullptr; }

int msa_sync(msa_ctx *c) {
    if (!c) return MSA_ERR_ARG;
    HIPC(c, join_side(c));
    HIPC(c, hipStreamSynchronize(c->stream));
    return MSA_OK;
}

int msa_load_csv(msa_ctx *c, const void *host, size_t n) {
    if (c) {
        c->fin_cache_n = 0;    // a new input
        c->dense_veto = false;  // a veto holds for the input that raised it
    }
    if (!c || (!host && n)) return MSA_ERR_ARG;
    HIPC(c, hipSetDevice(c->device));
    HIPC(c, join_side(c));
    HIPC(c, hipStreamSynchronize(c->stream));  // nothing in flight reads the old input
    HIPC(c, ensure(c->in_own, n + MSA_INPUT_PAD));
    if (n) HIPC(c, hipMemcpy(c->in_own.p, host, n, hipMemcpyHostToDevice));
    HIPC(c, hipMemset(c->in_own.as<char>() + n, 0, MSA_INPUT_PAD));
    HIPC(c, hipDeviceSynchronize());  // null-stream work: not ordered with the library's non-blocking streams
    c->in = c->in_own.as<u8>();
    c->n = n;
    c->in_base = c->in;
    c->n_base = n;
    c->stage = 0;
    return MSA_OK;
}

int msa_bind_csv(msa_ctx *c, const void *dev, size_t n) {
    if (!c || (!dev && n)) return MSA_ERR_ARG;
    c->fin_cache_n = 0;  // a new input
    c->dense_veto = false;  // a veto holds for the input that raised it
    HIPC(c, join_side(c));
    c->in = reinterpret_cast<const u8 *>(dev);
    c->n = n;
    c->in_base = c->in;
    c->n_base = n;
    c->stage = 0;
    return MSA_OK;
}

int msa_split_columns(msa_ctx *c, int flags) {
    if (!c) return MSA_ERR_ARG;
    HIPC(c, hipSetDevice(c->device));
    return do_split(c, flags);
}

int msa_count(msa_ctx *c) {
    if (!c) return MSA_ERR_ARG;
    HIPC(c, hipSetDevice(c->device));
    return do_count(c);
}

int msa_rank(msa_ctx *c) {
    if (!c) return MSA_ERR_ARG;
    HIPC(c, hipSetDevice(c->device));
    return do_rank(c);
}

int msa_run(msa_ctx *c, int flags) {
    if (!c) return MSA_ERR_ARG;
    HIPC(c, hipSetDevice(c->device));
    // overflowing tables grow inside each stage (do_split / do_count)
    int rc = do_split(c, flags);
    if (!rc) rc = do_count(c);
    if (!rc) rc = do_rank(c);
    const hipError_t e = join_side(c);  // a later sync on the library stream covers text.csv
    if (!rc && e != hipSuccess) rc = fail(c, MSA_ERR_HIP, "HIP error %s", hipGetErrorString(e));
    return rc;
}

int msa_get_summary(msa_ctx *c, msa_summary *out) {
    if (!c || !out) return MSA_ERR_ARG;
    if (c->stage < 1) return fail(c, MSA_ERR_ARG, "no results yet");
    *out = c->sum;
    return MSA_OK;
}

int msa_get_ranked(msa_ctx *c, int table, uint64_t first, uint64_t count, long long *counts, uint64_t *offsets,
                   char *keys, uint64_t keys_cap, uint64_t *keys_needed) {
    if (!c || (table != MSA_TABLE_WORDS && table != MSA_TABLE_ARTISTS)) return MSA_ERR_ARG;
    if (c->stage < 3) return fail(c, MSA_ERR_ARG, "msa_get_ranked before msa_rank");
    HIPC(c, hipSetDevice(c->device));
    Ranked &R = table == MSA_TABLE_WORDS ? c->rw : c->ra;
    int rc = fetch_ranked(c, R);
    if (rc) return rc;
    if (first > R.n) first = R.n;
    if (count > R.n - first) count = R.n - first;
    const u64 kb = R.h_off[first], ke = R.h_off[first + count];
    if (keys_needed) *keys_needed = ke - kb;
    if (keys && keys_cap < ke - kb) return fail(c, MSA_ERR_CAPACITY, "key buffer too small");
    for (u64 i = 0; i < count; ++i) {
        if (counts) counts[i] = (long long)R.h_counts[first + i];
        if (offsets) offsets[i] = R.h_off[first + i] - kb;
    }
    if (offsets) offsets[count] = ke - kb;
    if (keys && ke > kb) memcpy(keys, R.h_blob.data() + kb, ke - kb);
    return MSA_OK;
}

// tables up to this many lines (msa_ctx::csv_host_max) are written by the
// host loop: the device formatting's launches, scans and first-use
// allocations cost a small table more than the loop does
int msa_write_table_csv(msa_ctx *c, int table, const char *path, const char *key_header, int limit) {
    if (!c || !path || !key_header) return MSA_ERR_ARG;
    if (table != MSA_TABLE_WORDS && table != MSA_TABLE_ARTISTS) return MSA_ERR_ARG;
    if (c->stage < 3) return fail(c, MSA_ERR_ARG, "msa_write_table_csv before msa_rank");
    HIPC(c, hipSetDevice(c->device));
    Ranked &R = table == MSA_TABLE_WORDS ? c->rw : c->ra;
    u64 m = R.n;
    if (limit > 0 && (u64)limit < m) m = (u64)limit;
    if (m <= c->csv_host_max) {  // a small table: formatted on the host from the ranked arrays
        int rc = fetch_ranked(c, R);
        if (rc) return rc;
        FILE *fp = fopen(path, "w");
        if (!fp) return fail(c, MSA_ERR_IO, "Failed to open output file %s: %s", path, strerror(errno));
        std::string out = std::string(key_header) + ",count\n";
        char num[32];
        for (u64 i = 0; i < m; ++i) {
            out.push_back('"');
            for (u64 k = R.h_off[i]; k < R.h_off[i + 1]; ++k) {
                const char ch = R.h_blob[k];
                if (ch == '"') out.push_back('"');
                out.push_back(ch);
            }
            const int l = snprintf(num, sizeof num, "\",%lld\n", (long long)R.h_counts[i]);
            out.append(num, (size_t)l);
        }
        const bool ok = fwrite(out.data(), 1, out.size(), fp) == out.size();
        if (fclose(fp) != 0 || !ok) return fail(c, MSA_ERR_IO, "write failed: %s", path);
        return MSA_OK;
    }
    // a large one: the lines are formatted on the device from the ranked
    // arrays (k_csv_len, scan, k_csv_put) and written out in one pass (the
    // host loop had taken 2.4 s for configs[4]'s 50 M lines)
    u64 total = 0;
    if (m) {
        HIPC(c, ensure(c->csv_len, m * 8));
        HIPC(c, ensure(c->csv_pos, m * 8));
        HIPC(c, ensure(c->csv_bsum, ((m + 1023) / 1024 + 1) * 8));
        HIPC(c, ensure(c->small, 4096));
        u64 *d_total = reinterpret_cast<u64 *>(c->small.as<char>() + 3072);
        HIPC(c, msa_launch_csv_lines(0, R.off.as<u64>(), R.blob.as<u8>(), R.counts.as<u64>(), R.n, m, R.blob_len,
                                     table == MSA_TABLE_ARTISTS, c->csv_len.as<u64>(), c->csv_pos.as<u64>(),
                                     c->csv_bsum.as<u64>(), d_total, nullptr, c->stream));
        HIPC(c, hipMemcpyAsync(c->pin + kPinSmall, d_total, 8, hipMemcpyDeviceToHost, c->stream));
        HIPC(c, hipStreamSynchronize(c->stream));
        memcpy(&total, c->pin + kPinSmall, 8);
        HIPC(c, ensure(c->csv_out, total + 16));
        HIPC(c, msa_launch_csv_lines(1, R.off.as<u64>(), R.blob.as<u8>(), R.counts.as<u64>(), R.n, m, R.blob_len,
                                     table == MSA_TABLE_ARTISTS, c->csv_len.as<u64>(), c->csv_pos.as<u64>(),
                                     c->csv_bsum.as<u64>(), d_total, c->csv_out.as<u8>(), c->stream));
    }
    FILE *fp = fopen(path, "w");
    if (!fp) return fail(c, MSA_ERR_IO, "Failed to open output file %s: %s", path, strerror(errno));
    fprintf(fp, "%s,count\n", key_header);
    // a small file in one pageable copy; a large one through two pinned
    // halves, half k + 1 copied while half k is written (pinning them costs
    // ~20 ms once: not worth it for a few MB)
    static const u64 kHalf = 16ull << 20;
    bool ok = true;
    if (total && total <= kHalf) {
        std::vector<char> h(total);
        HIPC(c, hipMemcpyAsync(h.data(), c->csv_out.p, total, hipMemcpyDeviceToHost, c->stream));
        HIPC(c, hipStreamSynchronize(c->stream));
        ok = fwrite(h.data(), 1, total, fp) == total;
        total = 0;  // written
    }
    if (total && !c->csv_pin) HIPC(c, hipHostMalloc((void **)&c->csv_pin, 2 * kHalf, hipHostMallocDefault));
    auto half = [&](u64 k) { return c->csv_pin + (k & 1) * kHalf; };
    auto part = [&](u64 k) { return std::min<u64>(kHalf, total - k * kHalf); };
    const u64 nk = (total + kHalf - 1) / kHalf;
    if (nk) HIPC(c, hipMemcpyAsync(half(0), c->csv_out.as<u8>(), part(0), hipMemcpyDeviceToHost, c->stream));
    for (u64 k = 0; k < nk; ++k) {
        HIPC(c, hipStreamSynchronize(c->stream));  // half k is in
        if (k + 1 < nk)  // (its half was written out by the previous trip)
            HIPC(c, hipMemcpyAsync(half(k + 1), c->csv_out.as<u8>() + (k + 1) * kHalf, part(k + 1),
                                   hipMemcpyDeviceToHost, c->stream));
        ok = ok && fwrite(half(k), 1, part(k), fp) == part(k);
    }
    if (fclose(fp) != 0 || !ok) return fail(c, MSA_ERR_IO, "write failed: %s", path);
    return MSA_OK;
}

int msa_get_split_column(msa_ctx *c, int which, char **out, size_t *len) {
    if (!c || !out || !len || (which != 0 && which != 1)) return MSA_ERR_ARG;
    HIPC(c, join_side(c));  // text.csv (side stream) may still read the buffers this touches
    if (c->stage < 1) return fail(c, MSA_ERR_ARG, "msa_get_split_column before msa_split_columns");
    if (which == 1 && !c->have_tcol)
        return fail(c, MSA_ERR_ARG, "text column not materialised (pass MSA_SPLIT_TEXT_COLUMN)");
    HIPC(c, hipSetDevice(c->device));
    int rc;
    if ((rc = resolve_col_lens(c))) return rc;
    const u8 *b = which ? c->tcol.as<u8>() + c->tcol_off : c->acol.as<u8>();
    const u64 n = which ? c->tcol_len : c->acol_len;
    char *p = (char *)malloc(n + 1);
    if (!p) return fail(c, MSA_ERR_ARG, "out of host memory");
    HIPC(c, hipStreamSynchronize(c->stream));
    if (n) HIPC(c, hipMemcpy(p, b, n, hipMemcpyDeviceToHost));
    p[n] = 0;
    *out = p;
    *len = n;
    return MSA_OK;
}

int msa_set_artist_reader(msa_ctx *c, int exact) {
    if (!c) return MSA_ERR_ARG;
    c->artist_exact = exact != 0;
    return MSA_OK;
}

int msa_artist_reader_needed(msa_ctx *c, int *needed) {
    if (!c || !needed) return MSA_ERR_ARG;
    if (c->stage < 1) return fail(c, MSA_ERR_ARG, "msa_artist_reader_needed before msa_split_columns");
    HIPC(c, hipSetDevice(c->device));
    int rc;
    if ((rc = sync_counters(c))) return rc;
    *needed = (c->h_ctr.a_quoted || c->a_hdr_getline < c->a_hdr_len) ? 1 : 0;
    return MSA_OK;
}

int msa_set_profiling(msa_ctx *c, int on) {
    if (!c) return MSA_ERR_ARG;
    c->prof = on != 0;
    return MSA_OK;
}

int msa_get_profile(msa_ctx *c, msa_profile *out, int reset) {
    if (!c || !out) return MSA_ERR_ARG;
    HIPC(c, hipSetDevice(c->device));
    memset(out, 0, sizeof *out);
    for (int i = 0; i < ST_COUNT_ && i < MSA_PROF_MAX; ++i) {
        prof_harvest(c, i);
        ProfStage &s = c->ps[i];
        if (!s.launches) continue;
        const int k = out->n++;
        snprintf(out->name[k], sizeof out->name[k], "%s", kStageName[i]);
        out->ms[k] = s.ms;
        out->launches[k] = s.launches;
        out->bytes[k] = s.bytes;
        if (reset) { s.ms = 0; s.launches = 0; s.bytes = 0; }
    }
    return MSA_OK;
}

static_assert(sizeof(msa_fn_entry) == sizeof(FnEnt), "msa_fn_entry mirrors FnEnt");
static_assert(sizeof(msa_shard_fn) == sizeof(Fn), "msa_shard_fn mirrors Fn");

int msa_set_shard(msa_ctx *c, int first) {
    if (!c) return MSA_ERR_ARG;
    c->cont = first == 0;
    c->sharded = true;
    return MSA_OK;
}

// The raw piece: the loaded CSV shard, or this shard's artist.csv body.
static int piece_of(msa_ctx *c, int piece, const u8 **base, u64 *len) {
    if (piece == MSA_PIECE_CSV) {
        if (!c->in_base) return fail(c, MSA_ERR_ARG, "no input bound");
        *base = c->in_base;
        *len = c->n_base;
        return MSA_OK;
    }
    if (piece == MSA_PIECE_ARTISTS) {
        if (c->stage < 1) return fail(c, MSA_ERR_ARG, "artist piece before msa_split_columns");
        int rc;
        if ((rc = resolve_col_lens(c))) return rc;
        *base = c->acol.as<u8>() + c->a_hdr_getline;
        *len = c->acol_len - c->a_hdr_getline;
        return MSA_OK;
    }
    return fail(c, MSA_ERR_ARG, "bad piece %d", piece);
}

int msa_piece_size(msa_ctx *c, int piece, uint64_t *len) {
    if (!c || !len) return MSA_ERR_ARG;
    if (piece == MSA_PIECE_ARTISTS) HIPC(c, launch_artist_col(c));  // artist.csv read below; text.csv may keep running
    const u8 *base;
    u64 n;
    int rc;
    if ((rc = piece_of(c, piece, &base, &n))) return rc;
    *len = n;
    return MSA_OK;
}

int msa_shard_function(msa_ctx *c, int piece, msa_shard_fn *out) {
    if (!c || !out) return MSA_ERR_ARG;
    if (piece == MSA_PIECE_ARTISTS) HIPC(c, launch_artist_col(c));  // artist.csv read below; text.csv may keep running
    HIPC(c, hipSetDevice(c->device));
    const u8 *base;
    u64 len;
    int rc;
    if ((rc = piece_of(c, piece, &base, &len))) return rc;
    // msa_shard_head reads the earlier pieces' functions for the state at its
    // first byte: the quote parity p, the carried '\r' cr, and whether a record
    // starts exactly there (rs == the piece start).  Those depend only on the
    // piece's quote parity and its last bytes, so the function is built from
    // one parity reduction (a streaming read) instead of K1 + K2: for input
    // (p, cr), p' = p ^ q; the last byte b is read with parity p ^ q (b is no
    // '"' when it matters); cr' = b is an unquoted '\r'; a record starts at
    // the piece end iff b is an unquoted '\r' or '\n' -- unless the piece is
    // the single '\n' a carried '\r' swallows.  Record counts, c and z are
    // left 0 (unused by msa_shard_head).
    Fn f = fn_identity(0);
    if (len) {
        HIPC(c, ensure(c->small, 4096));
        u32 *d_q = reinterpret_cast<u32 *>(c->small.as<char>() + 3584);
        HIPC(c, msa_launch_quote_parity(base, len, d_q, c->stream));
        u32 q = 0;
        u8 last = 0;
        HIPC(c, hipMemcpyAsync(c->pin + kPinSmall, d_q, 4, hipMemcpyDeviceToHost, c->stream));
        HIPC(c, hipMemcpyAsync(c->pin + kPinSmall + 8, base + len - 1, 1, hipMemcpyDeviceToHost, c->stream));
        HIPC(c, hipStreamSynchronize(c->stream));
        memcpy(&q, c->pin + kPinSmall, 4);
        last = c->pin[kPinSmall + 8];
        q &= 1u;
        const bool term_byte = last == '\n' || last == '\r';
        for (u32 i = 0; i < 3; ++i) {
            const u32 p_in = i == 1, cr_in = i == 2;
            FnEnt &e = f.e[i];
            e.p = p_in ^ q;
            const bool unquoted = e.p == 0;
            e.cr = last == '\r' && unquoted;
            const bool ends = term_byte && unquoted && !(cr_in && len == 1 && last == '\n');
            e.has = ends;
            e.nterm = ends;
            e.rs = ends ? len : 0;
            e.c = 0;
            e.z = 0;
            e.pad = 0;
        }
    }
    memcpy(out, &f, sizeof f);
    return MSA_OK;
}

int msa_shard_head(msa_ctx *c, int piece, const msa_shard_fn *before, int nbefore, const uint64_t *sizes,
                   uint64_t *head) {
    if (!c || !head || nbefore < 0 || (nbefore && (!before || !sizes))) return MSA_ERR_ARG;
    if (piece == MSA_PIECE_ARTISTS) HIPC(c, launch_artist_col(c));  // artist.csv read below; text.csv may keep running
    HIPC(c, hipSetDevice(c->device));
    const u8 *base;
    u64 len;
    int rc;
    if ((rc = piece_of(c, piece, &base, &len))) return rc;
    // reader state at this piece's first byte: the earlier pieces' functions,
    // their record starts moved to global offsets, applied in order
    State s{0, 0, 0, 0, 0, 0};
    u64 g = 0;
    for (int q = 0; q < nbefore; ++q) {
        Fn f;
        memcpy(&f, &before[q], sizeof f);
        for (int i = 0; i < 3; ++i) f.e[i].rs += g;
        s = fn_apply(s, f);
        g += sizes[q];
    }
    *head = 0;
    if (!len || nbefore == 0) return MSA_OK;
    u8 b0 = 0;
    HIPC(c, hipMemcpy(&b0, base, 1, hipMemcpyDeviceToHost));
    if (s.cr && b0 == '\n') {  // the '\r' that ended the previous piece swallows this '\n'
        *head = 1;
        return MSA_OK;
    }
    if (s.rs == g) return MSA_OK;  // a record starts exactly here
    u64 *d_out = reinterpret_cast<u64 *>(c->small.as<char>() + 3072);
    HIPC(c, ensure(c->small, 4096));
    d_out = reinterpret_cast<u64 *>(c->small.as<char>() + 3072);
    HIPC(c, msa_launch_first_end(base, len, s.p, s.cr, d_out, c->stream));
    u64 v = len;
    HIPC(c, hipMemcpyAsync(&v, d_out, 8, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    *head = v;
    return MSA_OK;
}

int msa_segment_copy(msa_ctx *c, int piece, uint64_t off, uint64_t len, void *dst) {
    if (!c || (len && !dst)) return MSA_ERR_ARG;
    if (piece == MSA_PIECE_ARTISTS) HIPC(c, launch_artist_col(c));  // artist.csv read below; text.csv may keep running
    HIPC(c, hipSetDevice(c->device));
    const u8 *base;
    u64 plen;
    int rc;
    if ((rc = piece_of(c, piece, &base, &plen))) return rc;
    if (off > plen || len > plen - off) return fail(c, MSA_ERR_ARG, "segment out of range");
    if (len) HIPC(c, hipMemcpyAsync(dst, base + off, len, hipMemcpyDefault, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    return MSA_OK;
}

// Grow a device buffer keeping its first `keep` bytes.
static hipError_t grow_keep(DevBuf &b, size_t bytes, size_t keep, hipStream_t s) {
    if (b.cap >= bytes) return hipSuccess;
    void *np = nullptr;
    const size_t want = bytes + bytes / 4;
    hipError_t e = hipMalloc(&np, want);
    if (e != hipSuccess) return e;
    if (keep) e = hipMemcpyAsync(np, b.p, keep, hipMemcpyDeviceToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) { (void)hipFree(np); return e; }
    free_quiet(b.p);
    b.p = np;
    b.cap = want;
    return hipSuccess;
}

int msa_segment_set(msa_ctx *c, int piece, uint64_t skip, const void *tail, uint64_t tail_len) {
    if (!c || (tail_len && !tail)) return MSA_ERR_ARG;
    // the input is rewritten: text.csv (side stream) must be done with it
    HIPC(c, piece == MSA_PIECE_ARTISTS ? launch_artist_col(c) : join_side(c));
    HIPC(c, hipSetDevice(c->device));
    const u8 *base;
    u64 len;
    int rc;
    if ((rc = piece_of(c, piece, &base, &len))) return rc;
    if (skip > len) return fail(c, MSA_ERR_ARG, "skip beyond the piece");
    if (piece == MSA_PIECE_CSV) {
        if (tail_len && c->in_base != c->in_own.as<u8>())
            return fail(c, MSA_ERR_ARG, "appending to a bound (caller-owned) buffer; use msa_load_csv");
        if (tail_len) {
            HIPC(c, grow_keep(c->in_own, c->n_base + tail_len + MSA_INPUT_PAD, c->n_base, c->stream));
            c->in_base = c->in_own.as<u8>();
            HIPC(c, hipMemcpyAsync(c->in_own.as<u8>() + c->n_base, tail, tail_len, hipMemcpyDefault, c->stream));
        }
        if (c->in_base == c->in_own.as<u8>())
            HIPC(c, hipMemsetAsync(c->in_own.as<u8>() + c->n_base + tail_len, 0, MSA_INPUT_PAD, c->stream));
        c->in = c->in_base + skip;
        c->n = c->n_base - skip + tail_len;
        c->stage = 0;
    } else {
        const u64 b0 = c->a_hdr_getline;
        if (tail_len) {
            HIPC(c, grow_keep(c->acol, c->acol_len + tail_len + MSA_INPUT_PAD, c->acol_len, c->stream));
            HIPC(c, hipMemcpyAsync(c->acol.as<u8>() + c->acol_len, tail, tail_len, hipMemcpyDefault, c->stream));
        }
        HIPC(c, hipMemsetAsync(c->acol.as<u8>() + c->acol_len + tail_len, 0, MSA_INPUT_PAD, c->stream));
        c->a_beg = b0 + skip;
        c->a_end = c->acol_len + tail_len;
        c->artist_piece_set = true;  // the piece is read with the exact record reader
    }
    HIPC(c, hipStreamSynchronize(c->stream));
    return MSA_OK;
}

// ----------------------------------------------------------------- merge
static void fill_exp_src(msa_ctx *c, int table, ExpSrc &x, u64 *n) {
    memset(&x, 0, sizeof x);
    if (table == MSA_TABLE_ARTISTS) {
        x.artists = 1;
        x.a_tab = c->a_tab.as<u64>();
        x.a_list = c->a_list.as<u32>();
        x.na = c->h_ctr.a_claimed;
        x.arena = c->merged_a ? c->imp_a.as<u8>() : c->arena.as<u8>();
        x.key_off = c->key_off.as<u64>();
        x.key_len = c->key_len.as<u32>();
        *n = x.na;
        return;
    }
    x.s_tab = c->s_tab.as<u64>();
    x.s_list = c->s_list.as<u32>();
    x.ns = c->h_ctr.s_claimed;
    x.m_tab = c->m_tab.as<u64>();
    x.m_list = c->m_list.as<u32>();
    x.nm = c->h_ctr.m_claimed;
    x.l_tab = c->l_tab.as<u64>();
    x.l_list = c->l_list.as<u32>();
    x.nl = c->h_ctr.l_claimed;
    x.buf = c->merged_w ? c->imp_w.as<u8>() : c->in;
    x.extra = c->merged_w ? c->imp_w.as<u8>() : c->extra.as<u8>();
    x.l_pos = c->l_pos.as<u64>();
    x.l_len = c->l_len.as<u32>();
    if (c->dense_w && !c->merged_w) {  // the S / M words are the dense entries' planes
        x.d_K1 = c->rw.K[0][1].as<u64>();
        x.d_K0 = c->rw.K[0][2].as<u64>();
        x.d_cnt = c->rw.cnt.as<u64>();
        x.nd = x.ns + x.nm;  // (k_mb_dense counts its S and M entries into s_claimed / m_claimed)
        x.ns = x.nm = 0;
    }
    *n = x.nd + x.ns + x.nm + x.nl;
}

int msa_export_partitions(msa_ctx *c, int table, int nparts, uint64_t *part_bytes) {
    if (!c || nparts < 1 || nparts > 4096 || !part_bytes) return MSA_ERR_ARG;
    if (table != MSA_TABLE_WORDS && table != MSA_TABLE_ARTISTS) return MSA_ERR_ARG;
    if (c->stage < 2) return fail(c, MSA_ERR_ARG, "msa_export_partitions before msa_count");
    if (c->ranked_only & (table == MSA_TABLE_WORDS ? 1 : 2))
        return fail(c, MSA_ERR_ARG, "msa_export_partitions of a table merged by msa_import_ranked");
    // dense word entries are exported from their planes, which the ranking
    // reorders: before msa_rank only (the pipeline's merge comes before it)
    if (table == MSA_TABLE_WORDS && c->dense_w && !c->merged_w && c->stage >= 3)
        return fail(c, MSA_ERR_ARG, "msa_export_partitions of dense word entries after msa_rank");
    HIPC(c, hipSetDevice(c->device));
    ExpSrc x;
    u64 n;
    fill_exp_src(c, table, x, &n);
    const size_t P = (size_t)nparts;
    HIPC(c, ensure(c->exp_meta, 5 * P * 8));
    u64 *pcnt = c->exp_meta.as<u64>(), *pblob = pcnt + P, *pbase = pblob + P, *rcur = pbase + P, *bcur = rcur + P;
    HIPC(c, hipMemsetAsync(c->exp_meta.p, 0, 5 * P * 8, c->stream));
    HIPC(c, msa_launch_exp_count(x, n, (u32)P, pcnt, pblob, c->stream));
    std::vector<u64> h(2 * P), base(P);
    HIPC(c, hipMemcpyAsync(h.data(), pcnt, 2 * P * 8, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    u64 total = 0;
    for (size_t p = 0; p < P; ++p) {
        base[p] = total;
        part_bytes[p] = 32 + 32 * h[p] + h[P + p];
        total += part_bytes[p];
    }
    HIPC(c, ensure(c->exp_buf, total + 16));
    HIPC(c, hipMemcpyAsync(pbase, base.data(), P * 8, hipMemcpyHostToDevice, c->stream));
    HIPC(c, msa_launch_exp_write(x, n, (u32)P, pbase, pcnt, pblob, rcur, bcur, c->exp_buf.as<u8>(), c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    c->exp_bytes = total;
    return MSA_OK;
}

int msa_export_ranked(msa_ctx *c, int table, uint64_t limit, uint64_t *bytes) {
    if (!c || !bytes) return MSA_ERR_ARG;
    if (table != MSA_TABLE_WORDS && table != MSA_TABLE_ARTISTS) return MSA_ERR_ARG;
    if (c->stage < 3) return fail(c, MSA_ERR_ARG, "msa_export_ranked before msa_rank");
    HIPC(c, hipSetDevice(c->device));
    Ranked &R = table == MSA_TABLE_WORDS ? c->rw : c->ra;
    const u64 n = (limit && limit < R.n) ? limit : R.n;
    u64 end = R.blob_len;
    if (n < R.n) HIPC(c, hipMemcpy(&end, R.off.as<u64>() + n, 8, hipMemcpyDeviceToHost));
    if (end >> 32) return fail(c, MSA_ERR_CAPACITY, "ranked key blob over 4 GiB");
    const u64 total = 32 + 32 * n + end;
    HIPC(c, ensure(c->exp_buf, total + 16));
    HIPC(c, msa_launch_exp_ranked(R.counts.as<u64>(), R.off.as<u64>(), R.blob.as<u8>(), n, end, c->exp_buf.as<u8>(),
                                  c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    c->exp_bytes = total;
    *bytes = total;
    return MSA_OK;
}

int msa_export_copy(msa_ctx *c, void *dst) {
    if (!c || (c->exp_bytes && !dst)) return MSA_ERR_ARG;
    HIPC(c, hipSetDevice(c->device));
    if (c->exp_bytes) HIPC(c, hipMemcpyAsync(dst, c->exp_buf.p, c->exp_bytes, hipMemcpyDefault, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    return MSA_OK;
}

static int clear_one(msa_ctx *c, DevBuf &tab, DevBuf &list, u64 &used, u32 w) {
    if (used && tab.p) {
        hipLaunchKernelGGL(k_clear_slots, dim3((u32)((used + 255) / 256)), dim3(256), 0, c->stream, tab.as<u64>(),
                           list.as<u32>(), used, w);
        HIPC(c, hipGetLastError());
    }
    used = 0;
    return MSA_OK;
}

int msa_import_partitions(msa_ctx *c, int table, const void *src, const uint64_t *blk_off, int nblk) {
    if (!c || !blk_off || nblk < 1) return MSA_ERR_ARG;
    HIPC(c, launch_artist_col(c));  // it reads key_off / key_len, which an artist import rewrites
    if (table != MSA_TABLE_WORDS && table != MSA_TABLE_ARTISTS) return MSA_ERR_ARG;
    if (c->stage < 2) return fail(c, MSA_ERR_ARG, "msa_import_partitions before msa_count");
    HIPC(c, hipSetDevice(c->device));
    const bool art = table == MSA_TABLE_ARTISTS;
    const u64 total = blk_off[nblk];
    DevBuf &imp = art ? c->imp_a : c->imp_w;
    HIPC(c, ensure(imp, total + 64));
    if (total) HIPC(c, hipMemcpyAsync(imp.p, src, total, hipMemcpyDefault, c->stream));
    HIPC(c, ensure(c->imp_meta, (2 * (size_t)nblk + 2) * 8));
    u64 *d_off = c->imp_meta.as<u64>(), *d_base = d_off + nblk + 1;
    HIPC(c, hipMemcpyAsync(d_off, blk_off, ((size_t)nblk + 1) * 8, hipMemcpyHostToDevice, c->stream));
    const u64 rec_bound = total / 32 + 1;  // records are >= 32 bytes
    int rc;
    for (int attempt = 0; attempt < 8; ++attempt) {
        // fresh tables for this key partition; only this table's counters reset
        if (art) {
            if ((rc = clear_one(c, c->a_tab, c->a_list, c->a_used_prev, 4))) return rc;
        } else {
            if ((rc = clear_one(c, c->s_tab, c->s_list, c->s_used_prev, 2))) return rc;
            if ((rc = clear_one(c, c->m_tab, c->m_list, c->m_used_prev, 4))) return rc;
            if ((rc = clear_one(c, c->l_tab, c->l_list, c->lt_used_prev, 4))) return rc;
        }
        if ((rc = ensure_tables(c))) return rc;
        Counters *dc = c->ctr.as<Counters>();
        if (art) {
            HIPC(c, hipMemsetAsync(&dc->a_claimed, 0, 8, c->stream));
            HIPC(c, ensure(c->key_off, rec_bound * 8));
            HIPC(c, ensure(c->key_len, rec_bound * 4));
            HIPC(c, ensure(c->key_slot, rec_bound * 8));
        } else {
            HIPC(c, hipMemsetAsync(&dc->s_claimed, 0, 8, c->stream));
            HIPC(c, hipMemsetAsync(&dc->m_claimed, 0, 8, c->stream));
            HIPC(c, hipMemsetAsync(&dc->l_occ, 0, 8, c->stream));
            HIPC(c, hipMemsetAsync(&dc->l_claimed, 0, 8, c->stream));
        }
        HIPC(c, hipMemsetAsync(&dc->overflow, 0, 8, c->stream));
        HIPC(c, hipMemsetAsync(&dc->collision, 0, 8, c->stream));
        ImpDst d;
        memset(&d, 0, sizeof d);
        d.s_tab = c->s_tab.as<u64>(); d.s_mask = c->s_slots - 1; d.s_list = c->s_list.as<u32>(); d.s_list_cap = c->s_slots / 2;
        d.m_tab = c->m_tab.as<u64>(); d.m_mask = c->m_slots - 1; d.m_list = c->m_list.as<u32>(); d.m_list_cap = c->m_slots / 2;
        d.l_tab = c->l_tab.as<u64>(); d.l_mask = c->lt_slots - 1; d.l_list = c->l_list.as<u32>(); d.l_list_cap = c->lt_slots / 2;
        d.l_pos = c->l_pos.as<u64>(); d.l_len = c->l_len.as<u32>(); d.l_slot = c->l_slot.as<u64>(); d.l_cap = c->l_occ_cap;
        d.a_tab = c->a_tab.as<u64>(); d.a_mask = c->a_slots - 1; d.a_list = c->a_list.as<u32>(); d.a_list_cap = c->a_slots / 2;
        d.key_off = c->key_off.as<u64>(); d.key_len = c->key_len.as<u32>(); d.key_slot = c->key_slot.as<u64>();
        d.ctr = dc;
        d.artists = art ? 1 : 0;
        HIPC(c, msa_launch_imp(imp.as<u8>(), d_off, (u32)nblk, d_base, rec_bound, d, c->stream));
        if ((rc = sync_counters(c))) return rc;
        if (art) c->a_used_prev = std::min<u64>(c->h_ctr.a_claimed, c->a_slots / 2);
        else {
            c->s_used_prev = std::min<u64>(c->h_ctr.s_claimed, c->s_slots / 2);
            c->m_used_prev = std::min<u64>(c->h_ctr.m_claimed, c->m_slots / 2);
            c->lt_used_prev = std::min<u64>(c->h_ctr.l_claimed, c->lt_slots / 2);
        }
        if (c->h_ctr.overflow) {
            grow_tables(c);
            continue;
        }
        break;
    }
    if (c->h_ctr.overflow) return fail(c, MSA_ERR_CAPACITY, "merged table capacity overflow");
    // byte-exact collision checks of the hash-keyed entries
    u64 nrec_in = 0;
    HIPC(c, hipMemcpy(&nrec_in, d_base + nblk, 8, hipMemcpyDeviceToHost));
    if (art) {
        HIPC(c, msa_launch_artist_verify(imp.as<u8>(), c->key_off.as<u64>(), c->key_len.as<u32>(),
                                         c->key_slot.as<u64>(), nrec_in, c->a_tab.as<u64>(), c->ctr.as<Counters>(),
                                         c->stream));
    } else {
        const u64 nl = std::min<u64>(c->h_ctr.l_occ, c->l_occ_cap);
        HIPC(c, msa_launch_long_verify(imp.as<u8>(), imp.as<u8>(), c->l_pos.as<u64>(), c->l_len.as<u32>(),
                                       c->l_slot.as<u64>(), nl, c->l_tab.as<u64>(), c->ctr.as<Counters>(), c->stream));
    }
    if ((rc = sync_counters(c))) return rc;
    if (c->h_ctr.collision)
        return fail(c, MSA_ERR_COLLISION, "64-bit key hash collision detected while merging");
    c->ranked_only &= art ? ~2 : ~1;
    if (art) {
        c->merged_a = true;
        c->sum.n_artists = c->h_ctr.a_claimed;
    } else {
        c->merged_w = true;
        c->sum.n_words = c->h_ctr.s_claimed + c->h_ctr.m_claimed + c->h_ctr.l_claimed;
    }
    c->stage = 2;
    return MSA_OK;
}

}  // extern "C"

// ------------------------------------------------------------ diagnostics
// Not part of include/msa_hip.h: a run counter by name (tools/ablate.py).
extern "C" int msa_debug_stat(msa_ctx *c, const char *name, uint64_t *v) {
    if (!c || !name || !v) return MSA_ERR_ARG;
    int rc;
    if ((rc = sync_counters(c))) return rc;
    const Counters &k = c->h_ctr;
    const std::string n(name);
    if (n == "k3_misses") *v = k.k3_misses;
    else if (n == "dense") *v = c->dense_w ? 1 : 0;  // the last split wrote dense word entries
    else if (n == "dense_n") *v = k.dense_n;
    else if (n == "dense_veto") *v = c->dense_veto ? 1 : 0;
    else if (n == "total_words") *v = k.total_words;
    else if (n == "collision") *v = k.collision;
    else if (n == "a_long") *v = k.a_long;
    else if (n == "overflow") *v = k.overflow;
    else if (n == "span_fix") *v = k.span_fix;
    else if (n == "s_claimed") *v = k.s_claimed;
    else if (n == "m_claimed") *v = k.m_claimed;
    else if (n == "l_claimed") *v = k.l_claimed;
    else if (n == "split_attempts") *v = c->split_attempts;
    else if (n == "mlog_full") *v = k.mlog_full;
    else if (n == "s_table_used" || n == "m_table_used") {  // occupied slots, counted on the host
        const bool sm = n == "s_table_used";
        const u64 slots = sm ? c->s_slots : c->m_slots, w = sm ? 2 : 4;
        std::vector<u64> t(slots * w);
        if (slots) HIPC(c, hipMemcpy(t.data(), sm ? c->s_tab.p : c->m_tab.p, slots * w * 8, hipMemcpyDeviceToHost));
        u64 used = 0;
        for (u64 i = 0; i < slots; ++i) used += t[i * w] != 0;
        *v = used;
    }
    else return MSA_ERR_ARG;
    return MSA_OK;
}

// Root GPU of the final gather: the received blocks are the GPUs' ranked,
// disjoint key partitions (msa_export_ranked), merged into this context's
// ranking of the table by co-rank (csrc/msa_post.hip: k_mr_keys /
// k_mr_corank / k_mr_blob): O(n) scratch and no size limit.
int msa_import_ranked(msa_ctx *c, int table, const void *src, const uint64_t *blk_off, int nblk) {
    if (!c || !blk_off || nblk < 1) return MSA_ERR_ARG;
    if (table != MSA_TABLE_WORDS && table != MSA_TABLE_ARTISTS) return MSA_ERR_ARG;
    if (c->stage < 2) return fail(c, MSA_ERR_ARG, "msa_import_ranked before msa_count");
    HIPC(c, hipSetDevice(c->device));
    const bool art = table == MSA_TABLE_ARTISTS;
    Ranked &R = art ? c->ra : c->rw;
    const u64 total = blk_off[nblk];
    DevBuf &imp = art ? c->imp_a : c->imp_w;
    HIPC(c, ensure(imp, total + 64));
    if (total) HIPC(c, hipMemcpyAsync(imp.p, src, total, hipMemcpyDefault, c->stream));
    HIPC(c, ensure(c->imp_meta, (2 * (size_t)nblk + 2) * 8));
    u64 *d_off = c->imp_meta.as<u64>(), *d_base = d_off + nblk + 1;
    HIPC(c, hipMemcpyAsync(d_off, blk_off, ((size_t)nblk + 1) * 8, hipMemcpyHostToDevice, c->stream));
    ImpDst none;
    memset(&none, 0, sizeof none);
    HIPC(c, msa_launch_imp(imp.as<u8>(), d_off, (u32)nblk, d_base, 0, none, c->stream));  // record bases only
    std::vector<u64> base((size_t)nblk + 1);
    HIPC(c, hipMemcpyAsync(base.data(), d_base, base.size() * 8, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    const u64 n = base[nblk];
    if (n >> 32) return fail(c, MSA_ERR_CAPACITY, "merged table over 2^32 keys");
    // tiles: every block cut into runs of <= 1024 records (sorted, as the block is)
    std::vector<u64> ts;
    for (int p = 0; p < nblk; ++p)
        for (u64 s0 = base[p]; s0 < base[p + 1]; s0 += 1024) ts.push_back(s0);
    ts.push_back(n);
    const u32 T = (u32)(ts.size() - 1);
    for (int k = 0; k < 3; ++k) HIPC(c, ensure(R.K[1][k], std::max<u64>(n, 1) * 8));
    HIPC(c, ensure(R.K[2][0], ts.size() * 8));
    HIPC(c, ensure(R.ref, std::max<u64>(n, 1) * 8));
    HIPC(c, ensure(R.cnt, std::max<u64>(n, 1) * 8));
    HIPC(c, ensure(R.order, std::max<u64>(n, 1) * 4));
    HIPC(c, ensure(R.len, std::max<u64>(n, 1) * 8));
    HIPC(c, ensure(R.off, (n + 1) * 8));
    HIPC(c, ensure(R.counts, std::max<u64>(n, 1) * 8));
    HIPC(c, ensure(R.scan_bsum, ((n + 1023) / 1024 + 1) * 8));
    HIPC(c, ensure(c->blob_tot, 64));
    u64 *tot = c->blob_tot.as<u64>() + (art ? 1 : 0);
    HIPC(c, hipMemsetAsync(tot, 0, 8, c->stream));
    HIPC(c, hipMemcpyAsync(R.K[2][0].p, ts.data(), ts.size() * 8, hipMemcpyHostToDevice, c->stream));
    HIPC(c, msa_launch_merge_ranked(imp.as<u8>(), d_off, d_base, (u32)nblk, n, R.K[2][0].as<u64>(), T,
                                    R.K[1][0].as<u64>(), R.K[1][1].as<u64>(), R.K[1][2].as<u64>(), R.ref.as<u64>(),
                                    R.cnt.as<u64>(), R.order.as<u32>(), R.len.as<u64>(),
                                    R.off.as<u64>(), R.scan_bsum.as<u64>(), tot, c->stream));
    u64 blob = 0;
    HIPC(c, hipMemcpyAsync(c->pin + kPinSmall, tot, 8, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    memcpy(&blob, c->pin + kPinSmall, 8);
    HIPC(c, ensure(R.blob, blob + 16));
    HIPC(c, msa_launch_merge_blob(R.order.as<u32>(), n, imp.as<u8>(), R.ref.as<u64>(), R.cnt.as<u64>(),
                                  R.off.as<u64>(), R.blob.as<u8>(), R.counts.as<u64>(), c->stream));
    R.n = n;
    R.blob_len = blob;
    R.blob_cap = R.blob.cap - 16;
    R.blob_pending = false;
    R.host_valid = false;
    if (art) c->sum.n_artists = n;
    else c->sum.n_words = n;
    c->ranked_only |= art ? 2 : 1;
    c->stage = 3;
    return MSA_OK;
}

// Not part of include/msa_hip.h: the per-record arrays of the last split
// (diagnostics: kernel variants compared record by record).
extern "C" int msa_debug_records(msa_ctx *c, uint64_t *rec_start, uint32_t *nulrel, uint64_t cap, uint64_t *n) {
    if (!c || !n) return MSA_ERR_ARG;
    HIPC(c, join_side(c));  // text.csv (side stream) may still read the buffers this touches
    if (c->stage < 1) return MSA_ERR_ARG;
    HIPC(c, hipSetDevice(c->device));
    HIPC(c, hipStreamSynchronize(c->stream));
    *n = c->nrec;
    const u64 m = std::min<u64>(cap, c->nrec + 1);
    if (rec_start && m) HIPC(c, hipMemcpy(rec_start, c->rec_start.p, m * 8, hipMemcpyDeviceToHost));
    if (nulrel && m) HIPC(c, hipMemcpy(nulrel, c->nulrel.p, m * 4, hipMemcpyDeviceToHost));
    return MSA_OK;
}
