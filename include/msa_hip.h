/*
 * msa_hip.h -- C ABI of libmsa_hip, the MI355X (gfx950) implementation of the
 * Music-Analyst-AI hot path (/root/reference/src/parallel_spotify.c).
 *
 * Plain C: pointers, sizes and ints only -- no torch / HIP types cross this
 * boundary (streams are passed as `void *`, device buffers as `void *`).
 * Every entry point returns MSA_OK (0) or a negative MSA_ERR_* code; the
 * message of the last failure is available from msa_last_error().
 *
 * Which reference function each entry point replaces (file:line in
 * /root/reference/src/parallel_spotify.c):
 *
 *   msa_split_columns   read_csv_record 549-633, parse_csv_line 258-304,
 *                       duplicate_field 215-255, split_dataset_columns
 *                       640-721, header handling in main 788-827
 *   msa_count           the text / artist rank loops of main 853-999,
 *                       process_lyrics 350-394, ht_put 126-149
 *   msa_set_shard / msa_shard_function / msa_shard_head / msa_segment_*
 *                       (multi-GPU) the even byte split + re-sync of main
 *                       866-916, done exactly instead of at raw byte offsets
 *   msa_export_partitions / msa_export_ranked / msa_export_copy /
 *   msa_import_partitions
 *                       send_hash_table 397-410, receive_hash_table 413-432,
 *                       ht_merge 152-158, the merge loop of main 1011-1025
 *   msa_rank            ht_to_array 161-175 + qsort(entry_compare_desc)
 *                       178-188 inside write_table_csv 325-344
 *   msa_write_table_csv write_table_csv 325-344 / write_csv_entry 307-319
 *   msa_run             all of the above for one GPU
 */
#ifndef MSA_HIP_H
#define MSA_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MSA_ABI_VERSION 1

/* A device buffer handed to msa_bind_csv must stay readable this many bytes
 * past its logical end (vector loads run ahead; the bytes are ignored). */
#define MSA_INPUT_PAD 4096

enum {
    MSA_OK = 0,
    MSA_ERR_ARG = -1,        /* bad argument / call order                  */
    MSA_ERR_HIP = -2,        /* HIP runtime failure (no GPU, OOM, fault)   */
    MSA_ERR_NOHEADER = -3,   /* "Dataset does not contain a header row"    */
    MSA_ERR_BADHEADER = -4,  /* "Unable to parse dataset header"           */
    MSA_ERR_CAPACITY = -5,   /* a table or list overflowed its capacity     */
    MSA_ERR_COLLISION = -6,  /* 64-bit key-hash collision detected          */
    MSA_ERR_IO = -7,         /* file write failed                           */
    MSA_ERR_INPUT = -8       /* input the reference refuses (wcs: invalid   */
                             /* UTF-8, NUL, field limit, short row)         */
};

/* ---------------------------------------------------------------- corpus */

enum { MSA_GEN_ZIPF = 0, MSA_GEN_HIGHCARD = 1, MSA_GEN_TORTURE = 2 };

typedef struct {
    uint64_t seed;
    uint64_t n_songs;
    uint32_t vocab;          /* distinct lyric words (ZIPF/HIGHCARD)      */
    uint32_t n_artists;
    uint32_t words_per_song; /* mean lyric length in words                */
    int mode;                /* MSA_GEN_*                                 */
    int crlf;                /* 1: records end in "\r\n"                  */
} msa_gen_params;

/* Deterministic synthetic corpus; *out is malloc'ed, release with msa_free. */
int msa_gen_corpus(const msa_gen_params *p, char **out, size_t *len);
/* Songs [first_song, first_song + n_songs) of the corpus p describes (the
 * header row only when first_song is 0): the concatenation of consecutive
 * ranges is msa_gen_corpus's output.  ZIPF / HIGHCARD only.               */
int msa_gen_corpus_range(const msa_gen_params *p, uint64_t first_song, uint64_t n_songs, char **out, size_t *len);
void msa_free(void *p);
/* Identity of this build: the first 16 hex digits of the sha256 of the kernel
 * sources, headers and compile flags it was built from (the same for every
 * rebuild of the same sources).  PMC passes are stamped with it. */
const char *msa_build_id(void);

/* --------------------------------------------------------------- context */

typedef struct msa_ctx msa_ctx;

int msa_create(int device, msa_ctx **out);
void msa_destroy(msa_ctx *ctx);
const char *msa_last_error(const msa_ctx *ctx);
/* The HIP stream (hipStream_t) this context's work is ordered on.  text.csv
 * (MSA_SPLIT_TEXT_COLUMN) is written on a second, internal stream during the
 * ranking; msa_run and every entry point that reads it enqueue a wait for it
 * on this stream, so work queued here after msa_run -- and msa_sync -- sees
 * every result. */
void *msa_stream(msa_ctx *ctx);
int msa_sync(msa_ctx *ctx);

/* Input: copy a host CSV into context-owned HBM, or bind a caller-owned
 * device buffer (zero copy; MSA_INPUT_PAD readable bytes past n). */
int msa_load_csv(msa_ctx *ctx, const void *host_csv, size_t n);
int msa_bind_csv(msa_ctx *ctx, const void *dev_csv, size_t n);

/* ---------------------------------------------------------------- stages */

enum {
    MSA_SPLIT_TEXT_COLUMN = 1  /* also materialise text.csv (CLI output)    */
};

/* Header parse + record/field scan of the whole CSV in HBM + artist.csv
 * materialisation.  Word tokens of the lyric column are counted in the same
 * pass (the scan and the tokenizer share one read of the input). */
int msa_split_columns(msa_ctx *ctx, int flags);
/* Artist pass over the materialised artist column; finishes the counts. */
int msa_count(msa_ctx *ctx);
/* Rank both tables: count descending, ties by strcmp of the key bytes. */
int msa_rank(msa_ctx *ctx);
/* split + count + rank, single GPU; returns when results are on device. */
int msa_run(msa_ctx *ctx, int flags);

/* --------------------------------------------------------------- results */

typedef struct {
    long long total_songs;     /* records read from the artist column      */
    long long total_words;     /* tokens of length >= 3                    */
    uint64_t n_words;          /* distinct words                           */
    uint64_t n_artists;        /* distinct non-empty artist names          */
    uint64_t n_records;        /* CSV records incl. header                 */
    char artist_label[128];    /* header labels (parallel_spotify.c:810)   */
    char text_label[128];
    char artist_file[128];     /* sanitised split file base names          */
    char text_file[128];
} msa_summary;

int msa_get_summary(msa_ctx *ctx, msa_summary *out);

enum { MSA_TABLE_WORDS = 0, MSA_TABLE_ARTISTS = 1 };

/* Copy ranked entries [first, first+count) of a table to the host.
 * counts[i] = occurrences; key i is keys[offsets[i] .. offsets[i+1]).
 * offsets needs count+1 slots; keys needs keys_cap bytes (returns
 * MSA_ERR_CAPACITY and the needed size in *keys_needed when too small). */
int msa_get_ranked(msa_ctx *ctx, int table, uint64_t first, uint64_t count,
                   long long *counts, uint64_t *offsets, char *keys,
                   uint64_t keys_cap, uint64_t *keys_needed);

/* write_table_csv: "<key_header>,count" then "\"key\",count" lines
 * (quotes doubled), limit <= 0 means all entries. */
int msa_write_table_csv(msa_ctx *ctx, int table, const char *path,
                        const char *key_header, int limit);

/* Host copy of a materialised split column (0 = artist.csv, 1 = text.csv). */
int msa_get_split_column(msa_ctx *ctx, int which, char **out, size_t *len);

/* ------------------------------------------------------------- profiling
 * HIP-event timing of each pipeline stage on the context's stream (no
 * reference counterpart; the reference's MPI_Wtime bracketing lives in the
 * CLI).  Stage times accumulate over runs until read with reset != 0.     */
#define MSA_PROF_MAX 16
typedef struct {
    int n;                          /* stages with data                      */
    char name[MSA_PROF_MAX][32];
    double ms[MSA_PROF_MAX];        /* summed event time                     */
    uint64_t launches[MSA_PROF_MAX];/* how many times the stage ran          */
    uint64_t bytes[MSA_PROF_MAX];   /* summed algorithmic bytes  */
} msa_profile;

int msa_set_profiling(msa_ctx *ctx, int on);
int msa_get_profile(msa_ctx *ctx, msa_profile *out, int reset);

/* ------------------------------------------------- multi-GPU (one process
 * per GPU; the caller moves bytes between GPUs, e.g. with RCCL all-to-all).
 * A shard is a contiguous byte range of ONE logical CSV; shard 0 holds the
 * header row.  Replaces the reference's even byte split of the column files
 * plus per-rank re-synchronisation (parallel_spotify.c:866-916), which loses
 * or double-counts records at the cut points; here every record is processed
 * exactly once by the GPU whose shard holds its first byte.
 *
 *   1. msa_set_shard(ctx, rank == 0); msa_load_csv(ctx, shard)
 *   2. fn = msa_shard_function(ctx, MSA_PIECE_CSV)      -> all-gather the fns
 *   3. msa_shard_head(ctx, MSA_PIECE_CSV, fns[0..rank), sizes, &head)
 *      -> all-gather heads; a head (bytes of an earlier shard's last record)
 *         goes to the nearest earlier rank whose head < its size
 *   4. msa_segment_set(ctx, MSA_PIECE_CSV, head, tail)  (tail = later heads)
 *   5. msa_split_columns; then steps 2-4 again on MSA_PIECE_ARTISTS (the
 *      artist.csv reader may also carry state across pieces); msa_count
 *   6. msa_export_partitions / msa_export_copy -> all-to-all ->
 *      msa_import_partitions (words, artists); msa_rank ranks each GPU's
 *      key partition; the caller gathers the ranked partitions.            */

enum { MSA_PIECE_CSV = 0, MSA_PIECE_ARTISTS = 1 };

typedef struct {
    uint64_t nterm, rs;
    uint32_t p, cr, has, c, z, pad;
} msa_fn_entry;
/* Transfer function of a piece over the reader state (quote parity, pending
 * '\r', field commas, NUL, record count, open-record start). */
typedef struct {
    msa_fn_entry e[3];
} msa_shard_fn;

/* first != 0: this context holds shard 0 (with the header row). */
int msa_set_shard(msa_ctx *ctx, int first);
/* Bytes of the raw piece (the loaded shard / this shard's artist.csv body). */
int msa_piece_size(msa_ctx *ctx, int piece, uint64_t *len);
int msa_shard_function(msa_ctx *ctx, int piece, msa_shard_fn *out);
/* State after the pieces before this one (fns/sizes of ranks 0..nbefore-1)
 * -> number of leading bytes of this piece that belong to a record begun in
 * an earlier piece. */
int msa_shard_head(msa_ctx *ctx, int piece, const msa_shard_fn *before, int nbefore, const uint64_t *sizes,
                   uint64_t *head);
/* Copy bytes [off, off+len) of the raw piece to dst (host or device). */
int msa_segment_copy(msa_ctx *ctx, int piece, uint64_t off, uint64_t len, void *dst);
/* Process [skip, size) of the piece followed by tail (host or device bytes). */
int msa_segment_set(msa_ctx *ctx, int piece, uint64_t skip, const void *tail, uint64_t tail_len);

/* The artist pass (parallel_spotify.c:948-998) reads artist.csv with the
 * record reader.  When no accepted record's artist field holds a '"' outside
 * a quoted field (and the label has no '\n'), every artist.csv line is one
 * record and msa_count keys the lines directly.  msa_artist_reader_needed
 * reports (after msa_split_columns) whether that shortcut is unavailable;
 * msa_set_artist_reader(ctx, 1) forces the exact reader (a sharded run does
 * so on every rank when any rank needs it, then resolves MSA_PIECE_ARTISTS). */
int msa_artist_reader_needed(msa_ctx *ctx, int *needed);
int msa_set_artist_reader(msa_ctx *ctx, int exact);

/* Serialise the counted table as nparts key-hash partitions (wire format in
 * csrc/msa_merge.hip); part_bytes[p] = bytes of partition p's block.      */
int msa_export_partitions(msa_ctx *ctx, int table, int nparts, uint64_t *part_bytes);
/* After msa_rank: ranked entries [0, limit) of a table (all when limit is 0)
 * as ONE block of the same wire format.  A root GPU that imports every GPU's
 * block (msa_import_partitions, one block per GPU) and calls msa_rank holds
 * the global ranking -- or its top-limit: the key partitions are disjoint, so
 * the union of the per-GPU top-limit lists holds the global top-limit.
 * Replaces rank 0's receive + merge of every rank's table (main 1011-1025)
 * followed by the final qsort (write_table_csv 325-344).                    */
int msa_export_ranked(msa_ctx *ctx, int table, uint64_t limit, uint64_t *bytes);
/* Copy the last export (partitions or ranked block) to dst (host or device). */
int msa_export_copy(msa_ctx *ctx, void *dst);
/* Replace the table by the union of the received blocks (counts summed);
 * blk_off[0..nblk] are the blocks' byte offsets in src (last = total).     */
int msa_import_partitions(msa_ctx *ctx, int table, const void *src, const uint64_t *blk_off, int nblk);
/* Root GPU of the final gather: the blocks are every GPU's msa_export_ranked
 * block (ranked, disjoint key partitions); the table's ranking becomes their
 * k-way merge at any size (each key's global rank = its rank in its own block
 * + its co-ranks in the others; no re-insertion, no sort).  Replaces, with
 * msa_import_partitions + msa_rank, rank 0's merge + qsort (main 1011-1039).
 * A table merged this way is ranked-only until the next split or partition
 * import: msa_rank keeps its ranking, msa_export_partitions refuses it.     */
int msa_import_ranked(msa_ctx *ctx, int table, const void *src, const uint64_t *blk_off, int nblk);

/* ------------------------------------------- per-song word counter (row f)
 * The GPU path of /root/reference/scripts/word_count_per_song.py:
 *   msa_wcs_run          csv.DictReader over the "utf-8-sig" file (108-117,
 *                        delimiter ','), tokenize 28-38, process_row 91-99,
 *                        the Counter loops of main 124-139, most_common 145
 *   msa_wcs_get_csv /    the csv.writer outputs word_counts_global.csv and
 *   msa_wcs_write_outputs word_counts_by_song.csv (128-146)
 * Inputs the script fails on (invalid UTF-8, NUL, a field over 131072
 * characters, a row without artist/song/text) return MSA_ERR_INPUT; a header
 * without the three columns returns MSA_ERR_BADHEADER.                      */
typedef struct msa_wcs msa_wcs;
typedef struct {
    uint64_t total_rows;   /* data rows read ("Processadas N linhas")         */
    uint64_t song_rows;    /* rows with at least one token                    */
    uint64_t total_tokens; /* tokens counted                                  */
    uint64_t n_words;      /* distinct words = word_counts_global.csv lines   */
    uint64_t n_pairs;      /* word_counts_by_song.csv lines                   */
    uint64_t fallback_rows;/* rows the wave-per-window walk left to the       */
                           /* thread-per-row walk (long / unusual rows)       */
} msa_wcs_summary;
enum { MSA_WCS_GLOBAL = 0, MSA_WCS_BY_SONG = 1 };

int msa_wcs_create(int device, msa_wcs **out);
void msa_wcs_destroy(msa_wcs *w);
const char *msa_wcs_last_error(const msa_wcs *w);
void *msa_wcs_stream(msa_wcs *w);
int msa_wcs_load_csv(msa_wcs *w, const void *host_csv, size_t n);
/* The reader's field delimiter (default ','): the script's --delimiter, or
 * what csv.Sniffer guesses on its 65536-character sample (detect_delimiter,
 * word_count_per_song.py:42-49; split_csv_columns.py:48-66).  One ASCII
 * byte other than '"', CR, LF and NUL; MSA_ERR_ARG otherwise.  Also the
 * column splitter's writer delimiter (QUOTE_MINIMAL quoting).              */
int msa_wcs_set_delimiter(msa_wcs *w, int delimiter);
/* The column splitter's quoting: split_csv_columns.py's --quotechar
 * (90-95, used by detect_csv_params 48-66 for its reader and writer) and the
 * sniffed dialect's skipinitialspace (58).  quotechar: one ASCII byte other
 * than the delimiter, CR, LF and NUL (default '"').  msa_wcs_run (the
 * per-song counter, whose csv.DictReader reads the default dialect) refuses
 * anything but the default.                                                 */
int msa_wcs_set_quoting(msa_wcs *w, int quotechar, int skipinitialspace);
/* Delimiter, quotechar and skipinitialspace in one call, the pair validated
 * together (split_csv_columns.py's reader/writer dialect, 48-66, 90-95): a
 * quotechar equal to the OLD delimiter is fine here (e.g. --quotechar ','
 * with a sniffed ';'), which two separate calls would refuse.              */
int msa_wcs_set_dialect(msa_wcs *w, int delimiter, int quotechar, int skipinitialspace);
/* The scripts' --encoding (word_count_per_song.py:63-66,111;
 * split_csv_columns.py:97-101,130): utf8_sig = 1, "utf-8-sig" (default),
 * drops a leading BOM; 0, "utf-8", keeps it as the first field's first
 * character (U+FEFF in the first header name); 2, a single-byte
 * ASCII-compatible codec (latin-1, cp1252, ...: every byte one character,
 * decode + encode the identity, so the column splitter's bytes are the
 * script's; the host decodes the header names and refuses bytes the codec
 * leaves undefined): no UTF-8 check, no BOM handling; column splitter only
 * (msa_wcs_run fails with MSA_ERR_ARG).                                    */
int msa_wcs_set_encoding(msa_wcs *w, int utf8_sig);
/* log2 of the word-table slots of the next run (0 = sized from the input;
 * the table grows by itself when it fills). */
int msa_wcs_set_table_bits(msa_wcs *w, int bits);
int msa_wcs_run(msa_wcs *w);
int msa_wcs_get_summary(msa_wcs *w, msa_wcs_summary *out);
/* One output file's bytes (malloc'ed, release with msa_free). */
int msa_wcs_get_csv(msa_wcs *w, int which, char **out, size_t *len);
int msa_wcs_write_outputs(msa_wcs *w, const char *outdir);

/* Column splitter: the GPU part of /root/reference/scripts/split_csv_columns.py
 * (main 124-199) on the CSV loaded with msa_wcs_load_csv: csv.reader rows
 * (delimiter ',', quotechar '"'), every column's file body as csv.writer
 * writes it (lineterminator "\n", QUOTE_MINIMAL) -- rows after the header
 * (has_header != 0) or all rows.  ncols = fields of the first row.  The
 * column splitter and msa_wcs_run share the context: running one invalidates
 * the other's results.  MSA_ERR_NOHEADER = "CSV vazio.".                    */
int msa_csvcol_run(msa_wcs *w, int has_header, uint64_t *ncols, uint64_t *nrows);
/* Header field `col` of the first row (unescaped content), malloc'ed. */
int msa_csvcol_header(msa_wcs *w, uint64_t col, char **out, size_t *len);
/* Body bytes of column `col`'s file, malloc'ed (release with msa_free). */
int msa_csvcol_get(msa_wcs *w, uint64_t col, char **out, size_t *len);

#ifdef __cplusplus
}
#endif
#endif /* MSA_HIP_H */
