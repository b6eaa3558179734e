/*
 * parallel_spotify -- drop-in for the reference CLI
 * (/root/reference/src/parallel_spotify.c, main at 724-1113) running the hot
 * path on MI355X GPUs through libmsa_hip.
 *
 *   parallel_spotify <dataset.csv> [--word-limit N] [--artist-limit N]
 *                    [--output-dir DIR] [--device D] [--processes N | -np N]
 *
 * Writes, like the reference: DIR/split_columns/<artist>.csv and <text>.csv,
 * DIR/word_counts.csv, DIR/top_artists.csv, DIR/performance_metrics.json and
 * the same stdout summary.  The ranked CSVs are byte-identical to
 * `mpirun -np 1 bin/parallel_spotify` for ANY process count (the reference's
 * own results change with -np: its byte split loses or double-counts records
 * at the cut points; here every record is counted once).
 *
 * --processes N (N > 1), or N processes started by `mpirun -np N` (Hydra or
 * Open MPI, as the reference is launched): one process per GPU (GPUs
 * D .. D+N-1), the rank layer of msa_ranks.h in place of MPI.  Rank r reads bytes [r*n/N, (r+1)*n/N) of
 * the file, the ranks agree on exact record boundaries (shard transfer
 * functions, all-gathered), move the bytes of cut records to the rank where
 * they begin, split and count locally, merge the count tables by key-hash
 * partition (all-to-all), rank their partitions, and rank 0 gathers the
 * ranked partitions GPU-to-GPU and ranks their union (msa_export_ranked).
 * Transport: RCCL when every rank has its own GPU, else host shared memory
 * (several ranks on one GPU; MSA_TRANSPORT=rccl|shm overrides).  Each rank
 * writes its part of the split-column files at its offset.
 * performance_metrics.json: "processes": N and avg/min/max over the ranks,
 * as the reference reduces them (1077-1082).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <limits.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

#include "msa_hip.h"
#include "msa_ranks.h"

typedef struct {
    const char *dataset;
    int word_limit, artist_limit, device, processes;
    char outdir[PATH_MAX];
    char split_dir[PATH_MAX];
    /* bench mode (no reference counterpart; bench.py --driver chost): each
     * rank generates its song range of one synthetic corpus in memory
     * (msa_gen_corpus_range, bench.py's corpus) and times bench_steps runs of
     * the whole pipeline -- boundary exchange, split, count, merge, rank, full
     * ranked gather -- after bench_warmup untimed ones; no files are written */
    uint64_t synth_songs;
    uint64_t synth_seed;  /* --synthetic-seed (default 1) */
    int synth_mode;       /* --synthetic-mode zipf|highcard (configs[2]/[3] or configs[4]) */
    int bench_steps, bench_warmup;
} Opts;

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

/* ensure_directory_recursive (parallel_spotify.c:476-504) */
static int mkdirs(const char *path) {
    char b[PATH_MAX];
    size_t n = strlen(path);
    if (!n) return 0;
    if (n >= sizeof b) { errno = ENAMETOOLONG; return -1; }
    memcpy(b, path, n + 1);
    for (size_t i = 1; i < n; ++i)
        if (b[i] == '/' || b[i] == '\\') {
            char s = b[i];
            b[i] = 0;
            if (b[0] && strcmp(b, ".") && mkdir(b, 0777) != 0 && errno != EEXIST) { b[i] = s; return -1; }
            b[i] = s;
        }
    if (mkdir(b, 0777) != 0 && errno != EEXIST) return -1;
    return 0;
}

/* bytes [lo, hi) of a file (hi = SIZE_MAX: to the end) */
static char *read_range(const char *path, size_t lo, size_t hi, size_t *len) {
    int fd = open(path, O_RDONLY);
    if (fd < 0) return NULL;
    struct stat st;
    if (fstat(fd, &st) != 0) { close(fd); return NULL; }
    const size_t n = (size_t)st.st_size;
    if (hi > n) hi = n;
    if (lo > hi) lo = hi;
    char *p = (char *)malloc(hi - lo + 1);
    size_t got = 0;
    while (p && got < hi - lo) {
        ssize_t r = pread(fd, p + got, hi - lo - got, (off_t)(lo + got));
        if (r <= 0) { free(p); p = NULL; break; }
        got += (size_t)r;
    }
    close(fd);
    *len = got;
    return p;
}

static size_t file_size(const char *path, int *ok) {
    struct stat st;
    *ok = stat(path, &st) == 0;
    return *ok ? (size_t)st.st_size : 0;
}

static int write_at(const char *path, int create, uint64_t off, const char *p, size_t n) {
    int fd = open(path, O_WRONLY | (create ? O_CREAT | O_TRUNC : 0), 0666);
    if (fd < 0) return -1;
    size_t done = 0;
    while (done < n) {
        ssize_t w = pwrite(fd, p + done, n - done, (off_t)(off + done));
        if (w <= 0) { close(fd); return -1; }
        done += (size_t)w;
    }
    return close(fd);
}

static int fail_rc(msa_ctx *ctx, int rc, const char *what) {
    fprintf(stderr, "%s: %s\n", what, ctx ? msa_last_error(ctx) : "");
    return rc == MSA_ERR_NOHEADER || rc == MSA_ERR_BADHEADER ? EXIT_FAILURE : 2;
}

static void print_top(msa_ctx *ctx, int table, const char *fmt_suffix, const char *title) {
    msa_summary s;
    msa_get_summary(ctx, &s);
    uint64_t n = table == MSA_TABLE_WORDS ? s.n_words : s.n_artists;
    uint64_t k = n < 10 ? n : 10;
    long long counts[10];
    uint64_t offs[11], need = 0;
    char *keys = NULL;
    msa_get_ranked(ctx, table, 0, k, NULL, NULL, NULL, 0, &need);
    keys = (char *)malloc(need + 1);
    msa_get_ranked(ctx, table, 0, k, counts, offs, keys, need + 1, &need);
    printf("Top %zu %s:\n", (size_t)k, title);
    for (uint64_t i = 0; i < k; ++i) {
        printf("  %.*s: %lld%s\n", (int)(offs[i + 1] - offs[i]), keys + offs[i], counts[i], fmt_suffix);
    }
    free(keys);
}

/* word_counts.csv, top_artists.csv and the stdout summary (main 1027-1053) */
static void write_results(msa_ctx *ctx, const Opts *o, long long songs, long long words) {
    char path[PATH_MAX + 64];
    int rc;
    snprintf(path, sizeof path, "%s/word_counts.csv", o->outdir);
    if ((rc = msa_write_table_csv(ctx, MSA_TABLE_WORDS, path, "word", o->word_limit)))
        fprintf(stderr, "%s\n", msa_last_error(ctx));
    snprintf(path, sizeof path, "%s/top_artists.csv", o->outdir);
    if ((rc = msa_write_table_csv(ctx, MSA_TABLE_ARTISTS, path, "artist", o->artist_limit)))
        fprintf(stderr, "%s\n", msa_last_error(ctx));
    printf("=== Parallel Spotify Analysis ===\n");
    printf("Total songs processed: %lld\n", songs);
    printf("Total words counted: %lld\n", words);
    print_top(ctx, MSA_TABLE_WORDS, "", "words");
    print_top(ctx, MSA_TABLE_ARTISTS, " songs", "artists");
    fflush(stdout);
}

/* performance_metrics.json (main 1084-1108) */
static void write_metrics(const Opts *o, int procs, long long songs, long long words, const double *compute,
                          const double *total) {
    char path[PATH_MAX + 64];
    double cs = 0, cmin = compute[0], cmax = compute[0], ts = 0, tmin = total[0], tmax = total[0];
    for (int r = 0; r < procs; ++r) {
        cs += compute[r];
        ts += total[r];
        if (compute[r] < cmin) cmin = compute[r];
        if (compute[r] > cmax) cmax = compute[r];
        if (total[r] < tmin) tmin = total[r];
        if (total[r] > tmax) tmax = total[r];
    }
    snprintf(path, sizeof path, "%s/performance_metrics.json", o->outdir);
    FILE *mf = fopen(path, "w");
    if (!mf) {
        fprintf(stderr, "Failed to write performance metrics file\n");
        return;
    }
    fprintf(mf, "{\n");
    fprintf(mf, "  \"processes\": %d,\n", procs);
    fprintf(mf, "  \"total_songs\": %lld,\n", songs);
    fprintf(mf, "  \"total_words\": %lld,\n", words);
    fprintf(mf, "  \"compute_time\": {\n");
    fprintf(mf, "    \"avg_seconds\": %.6f,\n", cs / procs);
    fprintf(mf, "    \"min_seconds\": %.6f,\n", cmin);
    fprintf(mf, "    \"max_seconds\": %.6f\n", cmax);
    fprintf(mf, "  },\n");
    fprintf(mf, "  \"total_time\": {\n");
    fprintf(mf, "    \"avg_seconds\": %.6f,\n", ts / procs);
    fprintf(mf, "    \"min_seconds\": %.6f,\n", tmin);
    fprintf(mf, "    \"max_seconds\": %.6f\n", tmax);
    fprintf(mf, "  }\n");
    fprintf(mf, "}\n");
    fclose(mf);
}

/* ------------------------------------------------------------ one process */
static int run_single(const Opts *o) {
    size_t n = 0;
    char *csv = read_range(o->dataset, 0, SIZE_MAX, &n);
    if (!csv) { fprintf(stderr, "Failed to open dataset %s\n", o->dataset); return EXIT_FAILURE; }
    msa_ctx *ctx = NULL;
    int rc = msa_create(o->device, &ctx);
    if (rc) { fprintf(stderr, "libmsa_hip: cannot open GPU %d (code %d)\n", o->device, rc); return 2; }
    if ((rc = msa_load_csv(ctx, csv, n))) { rc = fail_rc(ctx, rc, "load"); goto out; }
    free(csv);
    csv = NULL;

    /* Timed region.  The reference brackets its text and artist passes
     * (parallel_spotify.c:850-851 .. 1000) for compute_time and the merge +
     * outputs for total_time (1068).  On the GPU the text pass (tokenising and
     * counting every lyric) runs inside the record/field scan of
     * msa_split_columns, so the clock starts before it; the split-column FILES
     * are written after the timed region (their bytes stay on the device
     * until then), as the reference writes them before its own. */
    double t0 = now_s();
    rc = msa_split_columns(ctx, MSA_SPLIT_TEXT_COLUMN);
    if (rc == MSA_ERR_NOHEADER) { rc = fail_rc(ctx, rc, "Dataset does not contain a header row"); goto out; }
    if (rc == MSA_ERR_BADHEADER) { rc = fail_rc(ctx, rc, "Unable to parse dataset header"); goto out; }
    if (rc) { rc = fail_rc(ctx, rc, "Failed to split dataset columns"); goto out; }
    if ((rc = msa_count(ctx)) || (rc = msa_sync(ctx))) { rc = fail_rc(ctx, rc, "count"); goto out; }
    double compute = now_s() - t0;
    if ((rc = msa_rank(ctx))) { rc = fail_rc(ctx, rc, "rank"); goto out; }
    msa_summary s;
    msa_get_summary(ctx, &s);
    write_results(ctx, o, s.total_songs, s.total_words);
    double total = now_s() - t0;

    for (int which = 0; which < 2; ++which) {
        char *col = NULL, path[PATH_MAX + 160];
        size_t cl = 0;
        if ((rc = msa_get_split_column(ctx, which, &col, &cl))) { rc = fail_rc(ctx, rc, "split column"); goto out; }
        snprintf(path, sizeof path, "%s/%s.csv", o->split_dir, which ? s.text_file : s.artist_file);
        if (write_at(path, 1, 0, col, cl) != 0) fprintf(stderr, "Failed to create split files in %s\n", o->split_dir);
        msa_free(col);
    }
    write_metrics(o, 1, s.total_songs, s.total_words, &compute, &total);
    rc = EXIT_SUCCESS;
out:
    free(csv);
    msa_destroy(ctx);
    return rc;
}

/* ------------------------------------------------------------ N processes */
typedef struct {
    msa_tr *t;
    msa_ctx *ctx;
} Rank;

#define TRY(x, what)                                        \
    do {                                                    \
        int rc_ = (x);                                      \
        if (rc_) return fail_rc(R->ctx, rc_, what);         \
    } while (0)
#define TRY_T(x, what)                                                         \
    do {                                                                       \
        if ((x)) {                                                             \
            fprintf(stderr, "rank %d: %s failed\n", R->t->rank, what);         \
            return 2;                                                          \
        }                                                                      \
    } while (0)

/* Exact record boundaries of a piece across the ranks (replaces the byte
 * split + re-synchronising reader of main 866-916): the pieces' transfer
 * functions are all-gathered, each rank finds the bytes at its start that
 * belong to a record begun earlier ("head") and sends them to the rank where
 * that record begins, which appends them to its piece. */
static int resolve_piece(Rank *R, int piece) {
    msa_tr *t = R->t;
    const int rank = t->rank, world = t->world;
    uint64_t size = 0, head = 0, sizes[MSA_MAX_RANKS], heads[MSA_MAX_RANKS], send[MSA_MAX_RANKS],
             recv[MSA_MAX_RANKS];
    msa_shard_fn fn, fns[MSA_MAX_RANKS];
    TRY(msa_piece_size(R->ctx, piece, &size), "piece size");
    TRY(msa_shard_function(R->ctx, piece, &fn), "shard function");
    TRY_T(t->allgather(t, &fn, sizeof fn, fns), "all-gather of shard functions");
    TRY_T(t->allgather(t, &size, sizeof size, sizes), "all-gather of piece sizes");
    if (rank > 0) TRY(msa_shard_head(R->ctx, piece, fns, rank, sizes, &head), "shard head");
    TRY_T(t->allgather(t, &head, sizeof head, heads), "all-gather of heads");
    msa_tail_plan(rank, heads, sizes, world, send, recv);
    uint64_t ns = 0, nr = 0;
    for (int p = 0; p < world; ++p) {
        ns += send[p];
        nr += recv[p];
    }
    void *sb = t->alloc(t, ns), *rb = t->alloc(t, nr);
    if (!sb || !rb) return 2;
    if (ns) TRY(msa_segment_copy(R->ctx, piece, 0, head, sb), "segment copy");
    TRY_T(t->alltoallv(t, sb, send, rb, recv), "head exchange");
    TRY(msa_segment_set(R->ctx, piece, head, nr ? rb : NULL, nr), "segment set");
    t->release(t, sb);
    t->release(t, rb);
    return 0;
}

/* Key-hash partition p of every rank's table goes to rank p, which imports
 * (sums) them: replaces send_hash_table / receive_hash_table (397-432). */
static int merge_table(Rank *R, int table) {
    msa_tr *t = R->t;
    const int world = t->world;
    uint64_t part[MSA_MAX_RANKS], all[MSA_MAX_RANKS * MSA_MAX_RANKS], recv[MSA_MAX_RANKS], off[MSA_MAX_RANKS + 1];
    TRY(msa_export_partitions(R->ctx, table, world, part), "export partitions");
    TRY_T(t->allgather(t, part, sizeof(uint64_t) * world, all), "all-gather of partition sizes");
    uint64_t ns = 0, nr = 0;
    off[0] = 0;
    for (int p = 0; p < world; ++p) {
        ns += part[p];
        recv[p] = all[p * world + t->rank];
        nr += recv[p];
        off[p + 1] = off[p] + recv[p];
    }
    void *sb = t->alloc(t, ns), *rb = t->alloc(t, nr);
    if (!sb || !rb) return 2;
    TRY(msa_export_copy(R->ctx, sb), "export copy");
    TRY_T(t->alltoallv(t, sb, part, rb, recv), "partition all-to-all");
    TRY(msa_import_partitions(R->ctx, table, rb, off, world), "import partitions");
    t->release(t, sb);
    t->release(t, rb);
    return 0;
}

/* Every rank's ranked partition (its top `limit`, or all) to rank 0, which
 * ranks their union: the global ranking (replaces the merge at 1011-1025 and
 * the qsort of write_table_csv). */
static int gather_ranked(Rank *R, const uint64_t *limit) {
    msa_tr *t = R->t;
    const int world = t->world;
    void *rb[2] = {NULL, NULL};
    uint64_t off[2][MSA_MAX_RANKS + 1];
    for (int table = 0; table < 2; ++table) {
        uint64_t bytes = 0, all[MSA_MAX_RANKS], send[MSA_MAX_RANKS] = {0}, recv[MSA_MAX_RANKS] = {0};
        TRY(msa_export_ranked(R->ctx, table, limit[table], &bytes), "export ranked");
        TRY_T(t->allgather(t, &bytes, sizeof bytes, all), "all-gather of ranked sizes");
        send[0] = bytes;
        uint64_t nr = 0;
        off[table][0] = 0;
        for (int p = 0; p < world; ++p) {
            if (t->rank == 0) recv[p] = all[p];
            nr += recv[p];
            off[table][p + 1] = off[table][p] + recv[p];
        }
        void *sb = t->alloc(t, bytes);
        rb[table] = t->alloc(t, nr);
        if (!sb || !rb[table]) return 2;
        TRY(msa_export_copy(R->ctx, sb), "export copy");
        TRY_T(t->alltoallv(t, sb, send, rb[table], recv), "ranked gather");
        t->release(t, sb);
    }
    if (t->rank == 0)  /* the k-way merge of the ranked, disjoint key partitions */
        for (int table = 0; table < 2; ++table)
            TRY(msa_import_ranked(R->ctx, table, rb[table], off[table], world), "import ranked");
    t->release(t, rb[0]);
    t->release(t, rb[1]);
    return 0;
}

/* One pipeline run of a rank (the timed unit of the bench mode): exact shard
 * boundaries, split, count, key-hash merge, ranking, full ranked gather. */
static int pipeline_step(Rank *R) {
    msa_tr *t = R->t;
    int rc;
    if ((rc = resolve_piece(R, MSA_PIECE_CSV))) return rc;
    if ((rc = msa_split_columns(R->ctx, MSA_SPLIT_TEXT_COLUMN))) return fail_rc(R->ctx, rc, "split");
    int need = 0;
    uint64_t need_any = 0;
    TRY(msa_artist_reader_needed(R->ctx, &need), "artist reader");
    TRY_T(msa_allreduce_sum_u64(t, (uint64_t)need, &need_any), "all-reduce");
    TRY(msa_set_artist_reader(R->ctx, need_any ? 1 : 0), "artist reader");
    if (need_any && (rc = resolve_piece(R, MSA_PIECE_ARTISTS))) return rc;
    TRY(msa_count(R->ctx), "count");
    if ((rc = merge_table(R, MSA_TABLE_WORDS)) || (rc = merge_table(R, MSA_TABLE_ARTISTS))) return rc;
    TRY(msa_rank(R->ctx), "rank");
    const uint64_t all[2] = {0, 0};
    return gather_ranked(R, all);
}

/* Bench mode: warmup + timed runs between barriers and device syncs; rank 0
 * prints one JSON line with the slowest rank's time and the corpus bytes. */
static int bench_ranks(Rank *R, const Opts *o, uint64_t nbytes) {
    msa_tr *t = R->t;
    int rc;
    for (int i = 0; i < o->bench_warmup; ++i)
        if ((rc = pipeline_step(R))) return rc;
    TRY(msa_set_profiling(R->ctx, 1), "profiling");
    msa_profile pr;
    TRY(msa_get_profile(R->ctx, &pr, 1), "profile");
    TRY(msa_sync(R->ctx), "sync");
    TRY_T(msa_barrier(t), "barrier");
    const double t0 = now_s();
    for (int i = 0; i < o->bench_steps; ++i)
        if ((rc = pipeline_step(R))) return rc;
    TRY(msa_sync(R->ctx), "sync");
    TRY_T(msa_barrier(t), "barrier");
    const double dt = now_s() - t0;
    TRY(msa_get_profile(R->ctx, &pr, 1), "profile");
    double all_dt[MSA_MAX_RANKS];
    uint64_t total = 0;
    TRY_T(t->allgather(t, &dt, sizeof dt, all_dt), "all-gather of timings");
    TRY_T(msa_allreduce_sum_u64(t, nbytes, &total), "all-reduce");
    if (t->rank == 0) {
        double mx = 0;
        for (int r = 0; r < t->world; ++r) mx = all_dt[r] > mx ? all_dt[r] : mx;
        printf("{\"driver\": \"chost\", \"ranks\": %d, \"steps\": %d, \"warmup\": %d, \"seconds\": %.6f, "
               "\"bytes_total\": %llu, \"bytes_rank0\": %llu, \"stages\": {",
               t->world, o->bench_steps, o->bench_warmup, mx, (unsigned long long)total,
               (unsigned long long)nbytes);
        for (int k = 0; k < pr.n; ++k)
            printf("%s\"%s\": [%.6f, %llu, %llu]", k ? ", " : "", pr.name[k], pr.ms[k],
                   (unsigned long long)pr.launches[k], (unsigned long long)pr.bytes[k]);
        printf("}}\n");
        fflush(stdout);
    }
    if (t->set_stream) t->set_stream(t, NULL);
    msa_destroy(R->ctx);
    t->destroy(t);
    return EXIT_SUCCESS;
}

static int rank_main(int rank, int world, msa_shared *sh, void *arg) {
    const Opts *o = (const Opts *)arg;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
        fprintf(stderr, "rank %d: no GPU\n", rank);
        return 2;
    }
    const int device = (o->device + rank) % ndev;
    const char *tk = getenv("MSA_TRANSPORT");
    const int use_rccl = tk ? strcmp(tk, "rccl") == 0 : ndev >= world;
    Rank RR = {NULL, NULL}, *R = &RR;
    R->t = use_rccl ? msa_tr_rccl(sh, rank, world, device) : msa_tr_shm(sh, rank, world);
    if (!R->t) return 2;
    msa_tr *t = R->t;

    size_t len = 0;
    char *part = NULL;
    if (o->synth_songs) {  /* bench mode: this rank's songs of the synthetic corpus */
        const msa_gen_params gp = {o->synth_seed, o->synth_songs, 50000, 5000, 30, o->synth_mode, 0};
        const uint64_t s0 = o->synth_songs * (uint64_t)rank / (uint64_t)world;
        const uint64_t s1 = o->synth_songs * (uint64_t)(rank + 1) / (uint64_t)world;
        if (msa_gen_corpus_range(&gp, s0, s1 - s0, &part, &len)) {
            fprintf(stderr, "rank %d: corpus generation failed\n", rank);
            return EXIT_FAILURE;
        }
    } else {
        int ok = 0;
        const size_t n = file_size(o->dataset, &ok);
        if (!ok) {
            if (rank == 0) fprintf(stderr, "Failed to open dataset %s\n", o->dataset);
            return EXIT_FAILURE;
        }
        const size_t lo = (size_t)((uint64_t)n * (uint64_t)rank / (uint64_t)world);
        const size_t hi = (size_t)((uint64_t)n * (uint64_t)(rank + 1) / (uint64_t)world);
        part = read_range(o->dataset, lo, hi, &len);
        if (!part) { fprintf(stderr, "rank %d: cannot read %s\n", rank, o->dataset); return EXIT_FAILURE; }
    }
    int rc = msa_create(device, &R->ctx);
    if (rc) { fprintf(stderr, "rank %d: libmsa_hip: cannot open GPU %d (code %d)\n", rank, device, rc); return 2; }
    /* RCCL exchanges on the library's stream: stream-ordered with the export /
     * import kernels around them (no host wait per exchange) */
    if (t->set_stream) t->set_stream(t, msa_stream(R->ctx));
    TRY(msa_set_shard(R->ctx, rank == 0), "set shard");
    TRY(msa_load_csv(R->ctx, part, len), "load");
    if (o->synth_songs) msa_free(part);
    else free(part);
    TRY_T(msa_barrier(t), "barrier");
    if (o->bench_steps > 0) return bench_ranks(R, o, (uint64_t)len);

    /* timed region as in run_single; compute = this rank's split + count */
    const double t0 = now_s();
    if ((rc = resolve_piece(R, MSA_PIECE_CSV))) return rc;
    rc = msa_split_columns(R->ctx, MSA_SPLIT_TEXT_COLUMN);
    if (rc == MSA_ERR_NOHEADER) return fail_rc(R->ctx, rc, "Dataset does not contain a header row");
    if (rc == MSA_ERR_BADHEADER) return fail_rc(R->ctx, rc, "Unable to parse dataset header");
    if (rc) return fail_rc(R->ctx, rc, "Failed to split dataset columns");
    /* the artist.csv lines are its records on every rank, unless some rank's
     * split says otherwise: then all read the artist pieces exactly */
    int need = 0;
    uint64_t need_any = 0;
    TRY(msa_artist_reader_needed(R->ctx, &need), "artist reader");
    TRY_T(msa_allreduce_sum_u64(t, (uint64_t)need, &need_any), "all-reduce");
    TRY(msa_set_artist_reader(R->ctx, need_any ? 1 : 0), "artist reader");
    if (need_any && (rc = resolve_piece(R, MSA_PIECE_ARTISTS))) return rc;
    TRY(msa_count(R->ctx), "count");
    TRY(msa_sync(R->ctx), "sync");
    const double compute = now_s() - t0;
    msa_summary s;
    TRY(msa_get_summary(R->ctx, &s), "summary");
    uint64_t songs = 0, words = 0;
    TRY_T(msa_allreduce_sum_u64(t, (uint64_t)s.total_songs, &songs), "all-reduce");
    TRY_T(msa_allreduce_sum_u64(t, (uint64_t)s.total_words, &words), "all-reduce");
    if ((rc = merge_table(R, MSA_TABLE_WORDS)) || (rc = merge_table(R, MSA_TABLE_ARTISTS))) return rc;
    TRY(msa_rank(R->ctx), "rank");
    /* the stdout summary needs the top 10 of each table */
    const uint64_t lim[2] = {o->word_limit > 0 ? (uint64_t)(o->word_limit > 10 ? o->word_limit : 10) : 0,
                             o->artist_limit > 0 ? (uint64_t)(o->artist_limit > 10 ? o->artist_limit : 10) : 0};
    if ((rc = gather_ranked(R, lim))) return rc;
    if (rank == 0) write_results(R->ctx, o, (long long)songs, (long long)words);
    TRY_T(msa_barrier(t), "barrier");
    const double total = now_s() - t0;

    /* split-column files: rank 0 names and creates them, every rank writes
     * its part at its offset (the concatenation of the ranks' columns in rank
     * order is the single-process column) */
    char names[2][128];
    memcpy(names[0], s.artist_file, 128);
    memcpy(names[1], s.text_file, 128);
    char all_names[MSA_MAX_RANKS][2][128];
    TRY_T(t->allgather(t, names, sizeof names, all_names), "all-gather of file names");
    for (int which = 0; which < 2; ++which) {
        char *col = NULL, path[PATH_MAX + 160];
        size_t cl = 0;
        uint64_t cls = 0, all_cl[MSA_MAX_RANKS], at = 0;
        TRY(msa_get_split_column(R->ctx, which, &col, &cl), "split column");
        cls = cl;
        TRY_T(t->allgather(t, &cls, sizeof cls, all_cl), "all-gather of column sizes");
        for (int r = 0; r < rank; ++r) at += all_cl[r];
        snprintf(path, sizeof path, "%s/%s.csv", o->split_dir, all_names[0][which]);
        int werr = 0;
        if (rank == 0) werr |= write_at(path, 1, 0, col, cl) != 0;
        TRY_T(msa_barrier(t), "barrier");
        if (rank > 0 && cl) werr |= write_at(path, 0, at, col, cl) != 0;
        if (werr) fprintf(stderr, "Failed to create split files in %s\n", o->split_dir);
        msa_free(col);
    }

    double all_c[MSA_MAX_RANKS], all_t[MSA_MAX_RANKS];
    TRY_T(t->allgather(t, &compute, sizeof compute, all_c), "all-gather of timings");
    TRY_T(t->allgather(t, &total, sizeof total, all_t), "all-gather of timings");
    if (rank == 0) write_metrics(o, world, (long long)songs, (long long)words, all_c, all_t);
    if (t->set_stream) t->set_stream(t, NULL);  /* the library's stream ends with its context */
    msa_destroy(R->ctx);
    t->destroy(t);
    return EXIT_SUCCESS;
}

int main(int argc, char **argv) {
    /* under `mpirun -np N` (the reference's launch, run_performance.sh:23)
     * this process is one of N ranks of one job */
    msa_launch L;
    const int launched = msa_launcher_detect(&L);
    if (launched < 0) {
        fprintf(stderr, "malformed MPI launcher environment (PMI_RANK/PMI_SIZE or OMPI_COMM_WORLD_RANK/SIZE)\n");
        return EXIT_FAILURE;
    }
    const int quiet = launched && L.rank != 0; /* messages once per job, as the reference's rank 0 */
    if (argc < 2) {
        if (quiet) return EXIT_FAILURE;
        fprintf(stderr,
                "Usage: %s <dataset.csv> [--word-limit N] [--artist-limit N] [--output-dir DIR] [--device D] "
                "[--processes N]\n",
                argv[0]);
        return EXIT_FAILURE;
    }
    Opts o;
    memset(&o, 0, sizeof o);
    o.dataset = argv[1];
    o.processes = 1;
    o.synth_seed = 1;
    o.synth_mode = MSA_GEN_ZIPF;
    snprintf(o.outdir, sizeof o.outdir, "output");
    for (int i = 2; i < argc; ++i) {
        if (!strcmp(argv[i], "--word-limit") && i + 1 < argc) o.word_limit = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--artist-limit") && i + 1 < argc) o.artist_limit = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--output-dir") && i + 1 < argc) {
            strncpy(o.outdir, argv[++i], sizeof o.outdir - 1);
            o.outdir[sizeof o.outdir - 1] = 0;
        } else if (!strcmp(argv[i], "--device") && i + 1 < argc) o.device = atoi(argv[++i]);
        else if ((!strcmp(argv[i], "--processes") || !strcmp(argv[i], "-np")) && i + 1 < argc)
            o.processes = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--synthetic-songs") && i + 1 < argc) o.synth_songs = strtoull(argv[++i], NULL, 10);
        else if (!strcmp(argv[i], "--synthetic-seed") && i + 1 < argc) o.synth_seed = strtoull(argv[++i], NULL, 10);
        else if (!strcmp(argv[i], "--synthetic-mode") && i + 1 < argc)
            o.synth_mode = !strcmp(argv[++i], "highcard") ? MSA_GEN_HIGHCARD : MSA_GEN_ZIPF;
        else if (!strcmp(argv[i], "--bench-steps") && i + 1 < argc) o.bench_steps = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--bench-warmup") && i + 1 < argc) o.bench_warmup = atoi(argv[++i]);
        else if (!quiet) fprintf(stderr, "Ignoring unknown argument: %s\n", argv[i]);
    }
    if (launched && L.world > 1 && o.processes != 1) {
        if (!quiet) fprintf(stderr, "--processes cannot be combined with the launcher's %d processes\n", L.world);
        return EXIT_FAILURE;
    }
    if (o.processes < 1 || o.processes > MSA_MAX_RANKS) {
        fprintf(stderr, "--processes must be in 1..%d\n", MSA_MAX_RANKS);
        return EXIT_FAILURE;
    }
    int l = snprintf(o.split_dir, sizeof o.split_dir, "%s/split_columns", o.outdir);
    if (l < 0 || (size_t)l >= sizeof o.split_dir) { fprintf(stderr, "Split directory path is too long\n"); return EXIT_FAILURE; }
    if (mkdirs(o.outdir) != 0) {
        fprintf(stderr, "Failed to prepare output directory %s: %s\n", o.outdir, strerror(errno));
        return EXIT_FAILURE;
    }
    if (mkdirs(o.split_dir) != 0) {
        fprintf(stderr, "Failed to prepare split directory %s: %s\n", o.split_dir, strerror(errno));
        return EXIT_FAILURE;
    }
    /* MSA_RANK_PATH=1 runs even one process through the rank layer (tests
     * the RCCL transport on a one-GPU box: a world of one) */
    const char *rp = getenv("MSA_RANK_PATH");
    if (o.bench_steps > 0 && !o.synth_songs) {
        fprintf(stderr, "--bench-steps needs --synthetic-songs\n");
        return EXIT_FAILURE;
    }
    if (launched && L.world > 1) return msa_launcher_run(&L, rank_main, &o);
    if (o.processes == 1 && !(rp && rp[0] == '1') && o.bench_steps <= 0) return run_single(&o);
    /* fork the ranks before anything initialises the GPU in this process */
    return msa_spawn_ranks(o.processes, rank_main, &o);
}
