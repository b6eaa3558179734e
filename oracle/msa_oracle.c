/*
 * msa_oracle.c -- CPU ORACLE (test infrastructure only).
 *
 * A single-process C restatement of the counting semantics of the reference
 * hot path, /root/reference/src/parallel_spotify.c (Music-Analyst-AI), for a
 * *virtual* MPI world size P.  The reference's results depend on P because it
 * cuts the split column files at raw byte offsets (parallel_spotify.c:866-882)
 * and re-synchronises each rank with a quote-unaware-of-history record read
 * (parallel_spotify.c:901-916); this file reproduces that exactly so the GPU
 * path can be checked against `mpirun -np P` for any P.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * run this program, and only as the checker.  It is never part of the product
 * path (libmsa_hip / parallel_spotify in music-analyst-ai_amd/).
 *
 * Parity pin: tests/test_oracle.py runs this oracle against the real
 * reference binary built from /root/reference by oracle/Makefile into
 * oracle/_ref/ (MPICH mpicc, `mpirun -np P`) on the committed golden inputs in
 * tests/golden/, and requires byte-identical word_counts.csv / top_artists.csv
 * and identical processes/total_songs/total_words.
 *
 * Usage: msa_oracle <csv> [--word-limit N] [--artist-limit N]
 *                   [--output-dir D] [--ranks P]
 */
#define _GNU_SOURCE
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <time.h>

typedef struct {
    unsigned char *p;
    size_t n, cap;
} Bytes;

static void die(const char *msg) {
    fprintf(stderr, "msa_oracle: %s\n", msg);
    exit(1);
}

static void bytes_put(Bytes *b, const void *src, size_t len) {
    if (b->n + len + 1 > b->cap) {
        size_t nc = b->cap ? b->cap : 4096;
        while (nc < b->n + len + 1) nc *= 2;
        b->p = (unsigned char *)realloc(b->p, nc);
        if (!b->p) die("out of memory");
        b->cap = nc;
    }
    memcpy(b->p + b->n, src, len);
    b->n += len;
    b->p[b->n] = 0;
}

/* C-locale ctype (the reference never calls setlocale). */
static int c_space(unsigned c) { return c == ' ' || (c >= 9 && c <= 13); }
static int c_alnum(unsigned c) {
    return (c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z');
}

/*
 * End (exclusive) of the CSV record that starts at `pos`.  Restates
 * read_csv_record (parallel_spotify.c:549-633): a '"' opens a quoted run,
 * '""' inside it is an escaped quote, an unquoted '\n' or '\r' ends the
 * record and a '\r' swallows one following '\n'.  Returns n if EOF ends it.
 */
static size_t record_end(const unsigned char *b, size_t n, size_t pos) {
    int q = 0;
    size_t i = pos;
    while (i < n) {
        unsigned c = b[i++];
        if (c == '"') {
            if (!q) q = 1;
            else if (i < n && b[i] == '"') i++;
            else q = 0;
        } else if (!q && (c == '\n' || c == '\r')) {
            if (c == '\r' && i < n && b[i] == '\n') i++;
            break;
        }
    }
    return i;
}

/* Length of the C string the reference sees for bytes [p, p+len): it stops at
 * the first NUL (strdup / strlen in parallel_spotify.c:263,216). */
static size_t cstr_len(const unsigned char *p, size_t len) {
    const void *z = memchr(p, 0, len);
    return z ? (size_t)((const unsigned char *)z - p) : len;
}

/* Strip trailing '\n'/'\r' (parallel_spotify.c:268-270 and 933-935). */
static size_t strip_eol(const unsigned char *p, size_t len) {
    while (len > 0 && (p[len - 1] == '\n' || p[len - 1] == '\r')) len--;
    return len;
}

/*
 * duplicate_field (parallel_spotify.c:215-255): trim C-locale whitespace; a
 * field that starts AND ends with '"' (and has >= 2 chars) is "quoted"; with
 * preserve_quotes the quoted span is copied raw, otherwise the outer quotes
 * are dropped and '""' pairs collapse to '"'; the result is trimmed again.
 */
static void dup_field(const unsigned char *f, size_t len, int preserve_quotes, Bytes *out) {
    out->n = 0;
    size_t s = 0, e = len;
    while (s < len && c_space(f[s])) s++;
    while (e > s && c_space(f[e - 1])) e--;
    int quoted = (e > s + 1 && f[s] == '"' && f[e - 1] == '"');
    unsigned char *tmp = (unsigned char *)malloc(e - s + 1);
    size_t j = 0;
    if (preserve_quotes && quoted) {
        memcpy(tmp, f + s, e - s);
        j = e - s;
    } else {
        size_t a = s, z = e;
        if (quoted) { a++; z--; }
        for (size_t i = a; i < z; ++i) {
            if (f[i] == '"' && i + 1 < z && f[i + 1] == '"') {
                tmp[j++] = '"';
                i++;
            } else {
                tmp[j++] = f[i];
            }
        }
    }
    size_t a = 0, z = j;
    while (a < z && c_space(tmp[a])) a++;
    while (z > a && c_space(tmp[z - 1])) z--;
    bytes_put(out, tmp + a, z - a);
    free(tmp);
}

/*
 * parse_csv_line (parallel_spotify.c:258-304): the record as a C string,
 * trailing EOL stripped, split at the first three commas outside quotes.
 * Field 0 is the artist, field 3 is "everything after the third comma".
 * Returns 0 (record skipped) when fewer than three such commas exist.
 */
static int split_record(const unsigned char *rec, size_t len, int preserve,
                        Bytes *artist, Bytes *text) {
    len = strip_eol(rec, cstr_len(rec, len));
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
    if (nc < 3) return 0;
    dup_field(rec, comma[0], preserve, artist);
    dup_field(rec + comma[2] + 1, len - comma[2] - 1, preserve, text);
    return 1;
}

/* ------------------------------------------------------------------------ */
/* string -> count table (open addressing); the oracle's own, not the ref's  */

typedef struct {
    char *key;
    size_t len;
    long long count;
} Slot;

typedef struct {
    Slot *s;
    size_t cap, used;
} Table;

static uint64_t h64(const unsigned char *p, size_t n) {
    uint64_t h = 0x9E3779B97F4A7C15ULL ^ n;
    for (size_t i = 0; i < n; ++i) {
        h ^= p[i];
        h *= 0x100000001B3ULL;
        h ^= h >> 29;
    }
    return h;
}

static void table_add(Table *t, const unsigned char *k, size_t n, long long delta);

static void table_grow(Table *t) {
    Table g = {0};
    g.cap = t->cap ? t->cap * 2 : 1024;
    g.s = (Slot *)calloc(g.cap, sizeof(Slot));
    if (!g.s) die("out of memory");
    for (size_t i = 0; i < t->cap; ++i)
        if (t->s[i].key) {
            size_t m = g.cap - 1, h = h64((unsigned char *)t->s[i].key, t->s[i].len) & m;
            while (g.s[h].key) h = (h + 1) & m;
            g.s[h] = t->s[i];
            g.used++;
        }
    free(t->s);
    *t = g;
}

static void table_add(Table *t, const unsigned char *k, size_t n, long long delta) {
    if ((t->used + 1) * 10 > t->cap * 7) table_grow(t);
    size_t m = t->cap - 1, h = h64(k, n) & m;
    while (t->s[h].key) {
        if (t->s[h].len == n && memcmp(t->s[h].key, k, n) == 0) {
            t->s[h].count += delta;
            return;
        }
        h = (h + 1) & m;
    }
    t->s[h].key = (char *)malloc(n + 1);
    memcpy(t->s[h].key, k, n);
    t->s[h].key[n] = 0;
    t->s[h].len = n;
    t->s[h].count = delta;
    t->used++;
}

/* Order of write_table_csv / entry_compare_desc (parallel_spotify.c:178-188):
 * larger count first, ties by strcmp (unsigned bytes). */
static int slot_cmp(const void *a, const void *b) {
    const Slot *x = (const Slot *)a, *y = (const Slot *)b;
    if (x->count != y->count) return x->count < y->count ? 1 : -1;
    return strcmp(x->key, y->key);
}

static Slot *table_sorted(const Table *t, size_t *out_n) {
    Slot *v = (Slot *)malloc(sizeof(Slot) * (t->used ? t->used : 1));
    size_t k = 0;
    for (size_t i = 0; i < t->cap; ++i)
        if (t->s[i].key) v[k++] = t->s[i];
    qsort(v, k, sizeof(Slot), slot_cmp);
    *out_n = k;
    return v;
}

/* ------------------------------------------------------------------------ */

/* Tokeniser of process_lyrics (parallel_spotify.c:350-394): maximal runs of
 * [A-Za-z0-9'] lower-cased; runs of length >= 3 are words. */
static void count_words(Table *words, const unsigned char *s, size_t n, long long *total) {
    unsigned char tok[4096];
    unsigned char *big = NULL;
    size_t len = 0, cap = sizeof tok;
    unsigned char *buf = tok;
    for (size_t i = 0; i <= n; ++i) {
        unsigned c = i < n ? s[i] : 0;
        if (i < n && (c_alnum(c) || c == '\'')) {
            if (len + 1 >= cap) {
                size_t nc = cap * 2;
                unsigned char *nb = (unsigned char *)malloc(nc);
                memcpy(nb, buf, len);
                if (big) free(big);
                big = buf = nb;
                cap = nc;
            }
            buf[len++] = (c >= 'A' && c <= 'Z') ? (unsigned char)(c + 32) : (unsigned char)c;
        } else if (len > 0) {
            if (len >= 3) {
                table_add(words, buf, len, 1);
                (*total)++;
            }
            len = 0;
        }
    }
    free(big);
}

/* compute_header_length (parallel_spotify.c:444-459): bytes up to and
 * including the first '\n' (getline), or the whole file if none. */
static size_t header_len(const Bytes *f) {
    const void *nl = memchr(f->p, '\n', f->n);
    return nl ? (size_t)((const unsigned char *)nl - f->p) + 1 : f->n;
}

/*
 * One rank's walk over a split column file (parallel_spotify.c:853-999):
 * even byte split of the data area, rank r>0 throws away the (partial)
 * record at its start offset, then reads whole records while the record
 * starts before its end offset (the last rank reads to EOF).
 */
typedef void (*RecordFn)(void *ctx, const unsigned char *rec, size_t len);

static void rank_walk(const Bytes *f, int rank, int P, RecordFn fn, void *ctx) {
    long long H = (long long)header_len(f);
    long long size = (long long)f->n;
    long long data = size > H ? size - H : 0;
    long long chunk = data / P, rem = data % P;
    long long start = H + rank * chunk + (rank < rem ? rank : rem);
    long long end = start + chunk + (rank < rem ? 1 : 0);
    if (rank == P - 1) end = size;
    size_t pos = (size_t)(start > H ? start : H);
    if (start > H && pos < f->n) pos = record_end(f->p, f->n, pos);
    while (pos < f->n) {
        if (rank != P - 1 && (long long)pos >= end) break;
        size_t e = record_end(f->p, f->n, pos);
        fn(ctx, f->p + pos, e - pos);
        pos = e;
    }
}

typedef struct {
    Table words, artists;
    long long total_words, total_songs;
    Bytes tmp;
} Counts;

static void on_text_record(void *vc, const unsigned char *rec, size_t len) {
    Counts *c = (Counts *)vc;
    len = strip_eol(rec, cstr_len(rec, len));
    dup_field(rec, len, 1, &c->tmp);
    if (c->tmp.n) count_words(&c->words, c->tmp.p, c->tmp.n, &c->total_words);
}

static void on_artist_record(void *vc, const unsigned char *rec, size_t len) {
    Counts *c = (Counts *)vc;
    len = strip_eol(rec, cstr_len(rec, len));
    dup_field(rec, len, 0, &c->tmp);
    if (c->tmp.n) table_add(&c->artists, c->tmp.p, c->tmp.n, 1);
    c->total_songs++;
}

/* sanitize_header_name (parallel_spotify.c:510-543), output <= 127 chars. */
static void sanitize(const Bytes *in, char *out) {
    size_t j = 0;
    for (size_t i = 0; i < in->n; ++i) {
        unsigned c = in->p[i];
        if (c == '\n' || c == '\r') continue;
        if (j + 1 >= 128) continue;
        if (c_space(c)) out[j++] = '_';
        else if (c_alnum(c) || c == '-' || c == '.' || c == '_') out[j++] = (char)c;
        else out[j++] = '_';
    }
    if (j == 0) { strcpy(out, "col"); return; }
    out[j] = 0;
}

static void write_csv(const char *path, const char *hdr, const Slot *v, size_t n, int limit) {
    FILE *fp = fopen(path, "w");
    if (!fp) { fprintf(stderr, "msa_oracle: cannot write %s\n", path); return; }
    fprintf(fp, "%s,count\n", hdr);
    size_t m = (limit > 0 && (size_t)limit < n) ? (size_t)limit : n;
    for (size_t i = 0; i < m; ++i) {
        fputc('"', fp);
        for (const char *p = v[i].key; *p; ++p) {
            if (*p == '"') fputc('"', fp);
            fputc(*p, fp);
        }
        fprintf(fp, "\",%lld\n", v[i].count);
    }
    fclose(fp);
}

static void mkdirs(const char *path) {
    char b[4096];
    size_t n = strlen(path);
    if (n >= sizeof b) die("path too long");
    memcpy(b, path, n + 1);
    for (size_t i = 1; i < n; ++i)
        if (b[i] == '/') { b[i] = 0; mkdir(b, 0777); b[i] = '/'; }
    mkdir(b, 0777);
}

static void write_file(const char *path, const Bytes *b) {
    FILE *fp = fopen(path, "wb");
    if (!fp) { fprintf(stderr, "msa_oracle: cannot write %s\n", path); return; }
    if (b->n) fwrite(b->p, 1, b->n, fp);
    fclose(fp);
}

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s <csv> [--word-limit N] [--artist-limit N] [--output-dir D] [--ranks P]\n", argv[0]);
        return 1;
    }
    const char *csv = argv[1], *outdir = "output";
    int word_limit = 0, artist_limit = 0, P = 1;
    for (int i = 2; i < argc; ++i) {
        if (!strcmp(argv[i], "--word-limit") && i + 1 < argc) word_limit = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--artist-limit") && i + 1 < argc) artist_limit = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--output-dir") && i + 1 < argc) outdir = argv[++i];
        else if (!strcmp(argv[i], "--ranks") && i + 1 < argc) P = atoi(argv[++i]);
        else fprintf(stderr, "Ignoring unknown argument: %s\n", argv[i]);
    }
    if (P < 1) P = 1;

    Bytes in = {0};
    FILE *fp = fopen(csv, "rb");
    if (!fp) die("cannot open dataset");
    unsigned char blk[1 << 16];
    size_t got;
    while ((got = fread(blk, 1, sizeof blk, fp)) > 0) bytes_put(&in, blk, got);
    fclose(fp);
    if (!in.p) bytes_put(&in, "", 0);

    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);

    /* Header (parallel_spotify.c:788-819). */
    if (in.n == 0) die("Dataset does not contain a header row");
    size_t hend = record_end(in.p, in.n, 0);
    Bytes hart = {0}, htxt = {0};
    if (!split_record(in.p, hend, 0, &hart, &htxt)) die("Unable to parse dataset header");
    char alabel[128] = {0}, tlabel[128] = {0}, aname[128], tname[128];
    memcpy(alabel, hart.p ? (char *)hart.p : "", hart.n < 127 ? hart.n : 127);
    memcpy(tlabel, htxt.p ? (char *)htxt.p : "", htxt.n < 127 ? htxt.n : 127);
    alabel[strnlen(alabel, 127)] = 0;
    tlabel[strnlen(tlabel, 127)] = 0;
    sanitize(&hart, aname);
    sanitize(&htxt, tname);

    /* Column split (parallel_spotify.c:640-721). */
    Bytes acol = {0}, tcol = {0}, fa = {0}, ft = {0};
    const char *ah = *alabel ? alabel : "Artists", *th = *tlabel ? tlabel : "Texts";
    bytes_put(&acol, ah, strlen(ah));
    bytes_put(&acol, "\n", 1);
    bytes_put(&tcol, th, strlen(th));
    bytes_put(&tcol, "\n", 1);
    for (size_t pos = hend; pos < in.n;) {
        size_t e = record_end(in.p, in.n, pos);
        if (split_record(in.p + pos, e - pos, 1, &fa, &ft)) {
            bytes_put(&acol, fa.p ? fa.p : (unsigned char *)"", fa.n);
            bytes_put(&acol, "\n", 1);
            bytes_put(&tcol, ft.p ? ft.p : (unsigned char *)"", ft.n);
            bytes_put(&tcol, "\n", 1);
        }
        pos = e;
    }

    /* P virtual ranks over the two column files, merged like ranks 1..P-1
     * sending to rank 0 (parallel_spotify.c:1011-1025). */
    Counts c = {0};
    for (int r = 0; r < P; ++r) {
        rank_walk(&tcol, r, P, on_text_record, &c);
        rank_walk(&acol, r, P, on_artist_record, &c);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    double secs = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);

    char path[4096];
    mkdirs(outdir);
    snprintf(path, sizeof path, "%s/split_columns", outdir);
    mkdirs(path);
    snprintf(path, sizeof path, "%s/split_columns/%s.csv", outdir, aname);
    write_file(path, &acol);
    snprintf(path, sizeof path, "%s/split_columns/%s.csv", outdir, tname);
    write_file(path, &tcol);

    size_t nw, na;
    Slot *w = table_sorted(&c.words, &nw);
    Slot *a = table_sorted(&c.artists, &na);
    snprintf(path, sizeof path, "%s/word_counts.csv", outdir);
    write_csv(path, "word", w, nw, word_limit);
    snprintf(path, sizeof path, "%s/top_artists.csv", outdir);
    write_csv(path, "artist", a, na, artist_limit);

    printf("=== Parallel Spotify Analysis ===\n");
    printf("Total songs processed: %lld\n", c.total_songs);
    printf("Total words counted: %lld\n", c.total_words);
    size_t pw = nw < 10 ? nw : 10, pa = na < 10 ? na : 10;
    printf("Top %zu words:\n", pw);
    for (size_t i = 0; i < pw; ++i) printf("  %s: %lld\n", w[i].key, w[i].count);
    printf("Top %zu artists:\n", pa);
    for (size_t i = 0; i < pa; ++i) printf("  %s: %lld songs\n", a[i].key, a[i].count);

    snprintf(path, sizeof path, "%s/performance_metrics.json", outdir);
    FILE *mf = fopen(path, "w");
    if (mf) {
        fprintf(mf, "{\n  \"processes\": %d,\n  \"total_songs\": %lld,\n  \"total_words\": %lld,\n", P,
                c.total_songs, c.total_words);
        fprintf(mf, "  \"compute_time\": {\n    \"avg_seconds\": %.6f,\n    \"min_seconds\": %.6f,\n"
                    "    \"max_seconds\": %.6f\n  },\n", secs, secs, secs);
        fprintf(mf, "  \"total_time\": {\n    \"avg_seconds\": %.6f,\n    \"min_seconds\": %.6f,\n"
                    "    \"max_seconds\": %.6f\n  }\n}\n", secs, secs, secs);
        fclose(mf);
    }
    return 0;
}
