/*
 * msa_gen.c -- deterministic synthetic Spotify-Million-Song-shaped corpora.
 *
 * The real spotify_millsongdata.csv is not available (the reference lists it
 * in .MISSING_LARGE_BLOBS), so every workload is generated.  The shape follows
 * what /root/reference/src/parallel_spotify.c consumes: header
 * `artist,song,link,text`, an artist field (sometimes quoted because it holds
 * a comma), a song title, a link, and the lyrics as a quoted multi-line field
 * whose lines end in "  \n" and that may carry escaped quotes ("").
 *
 * Modes (BASELINE.json configs):
 *   MSA_GEN_ZIPF        configs[2]/[3]: Zipfian vocabulary lyrics
 *   MSA_GEN_HIGHCARD    configs[4]: high-cardinality tokens, skewed artists,
 *                       long tokens that leave the short-key fast path
 *   MSA_GEN_TORTURE     CSV-syntax torture (quotes, commas, CR, CRLF, NUL,
 *                       unquoted fields with stray quotes) for parity tests
 *
 * Same (params) -> same bytes, on every machine.  Pure host C, no HIP.
 * ZIPF / HIGHCARD songs are independent draws (per-song generator state), so
 * msa_gen_corpus_range produces any song range of a corpus -- each GPU of
 * configs[3] generates only its own shard -- and large ranges are generated
 * on several host threads.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "msa_hip.h"

typedef struct {
    uint64_t s;
} Rng;

static inline uint64_t rng_next(Rng *r) {
    uint64_t z = (r->s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static inline uint32_t rng_below(Rng *r, uint32_t n) {
    return (uint32_t)(((rng_next(r) >> 32) * (uint64_t)n) >> 32);
}
static inline double rng_unit(Rng *r) { return (rng_next(r) >> 11) * (1.0 / 9007199254740992.0); }

typedef struct {
    char *p;
    size_t n, cap;
    int oom;
} Out;

static void out_reserve(Out *o, size_t extra) {
    if (o->n + extra <= o->cap) return;
    size_t nc = o->cap ? o->cap : (1u << 20);
    while (nc < o->n + extra) nc *= 2;
    char *np = (char *)realloc(o->p, nc);
    if (!np) { o->oom = 1; return; }
    o->p = np;
    o->cap = nc;
}
static inline void out_put(Out *o, const char *s, size_t n) {
    out_reserve(o, n);
    if (o->oom) return;
    memcpy(o->p + o->n, s, n);
    o->n += n;
}
static inline void out_c(Out *o, char c) { out_put(o, &c, 1); }
static inline void out_s(Out *o, const char *s) { out_put(o, s, strlen(s)); }

/* Walker alias table for O(1) Zipf draws. */
typedef struct {
    uint32_t n;
    double *prob;
    uint32_t *alias;
} Alias;

static int alias_build(Alias *a, uint32_t n, double s) {
    a->n = n;
    a->prob = (double *)malloc(sizeof(double) * n);
    a->alias = (uint32_t *)malloc(sizeof(uint32_t) * n);
    double *w = (double *)malloc(sizeof(double) * n);
    uint32_t *small = (uint32_t *)malloc(sizeof(uint32_t) * n), *large = (uint32_t *)malloc(sizeof(uint32_t) * n);
    if (!a->prob || !a->alias || !w || !small || !large) return -1;
    double tot = 0;
    for (uint32_t i = 0; i < n; ++i) {
        double x = 1.0, b = (double)(i + 1);
        /* x = b^-s without libm: exp(-s*ln b) via repeated sqrt-free series is
         * overkill; use the integer-friendly form for s in {1.0, 1.1}. */
        if (s == 1.0) x = 1.0 / b;
        else {
            double l = 0, y = b; /* ln(b) by argument reduction */
            while (y > 2.0) { y *= 0.5; l += 0.6931471805599453; }
            double t = (y - 1) / (y + 1), t2 = t * t, sum = 0, term = t;
            for (int k = 1; k < 40; k += 2) { sum += term / k; term *= t2; }
            l += 2 * sum;
            double e = -s * l, r = 1, tt = 1; /* exp(e) */
            int sh = 0;
            while (e < -1) { e *= 0.5; sh++; }
            for (int k = 1; k < 30; ++k) { tt *= e / k; r += tt; }
            while (sh--) r *= r;
            x = r;
        }
        w[i] = x;
        tot += x;
    }
    uint32_t ns = 0, nl = 0;
    for (uint32_t i = 0; i < n; ++i) {
        w[i] = w[i] * n / tot;
        if (w[i] < 1.0) small[ns++] = i; else large[nl++] = i;
    }
    while (ns && nl) {
        uint32_t s_ = small[--ns], l_ = large[--nl];
        a->prob[s_] = w[s_];
        a->alias[s_] = l_;
        w[l_] = (w[l_] + w[s_]) - 1.0;
        if (w[l_] < 1.0) small[ns++] = l_; else large[nl++] = l_;
    }
    while (nl) { uint32_t l_ = large[--nl]; a->prob[l_] = 1.0; a->alias[l_] = l_; }
    while (ns) { uint32_t s_ = small[--ns]; a->prob[s_] = 1.0; a->alias[s_] = s_; }
    free(w);
    free(small);
    free(large);
    return 0;
}
static inline uint32_t alias_draw(const Alias *a, Rng *r) {
    uint32_t i = rng_below(r, a->n);
    return rng_unit(r) < a->prob[i] ? i : a->alias[i];
}
static void alias_free(Alias *a) {
    free(a->prob);
    free(a->alias);
}

static const char *HEAD_WORDS[] = {
    "the", "you", "i", "to", "and", "a", "me", "my", "it", "in", "of", "your", "that", "on", "is",
    "love", "all", "be", "we", "for", "don't", "i'm", "so", "know", "no", "with", "just", "oh", "but",
    "like", "this", "baby", "got", "when", "can", "what", "now", "get", "up", "go", "will", "down",
    "never", "can't", "one", "out", "heart", "yeah", "let", "see", "do", "time", "it's", "want", "feel",
    "come", "way", "say", "are", "there", "they", "back", "take", "make", "if", "she", "he", "night",
    "life", "was", "world", "girl", "good", "give", "need", "how", "think", "where", "day", "tell",
    "away", "right", "gonna", "cause", "from", "again", "eyes", "more", "won't", "nothing", "ever",
    "only", "wanna", "still", "hold", "home", "dream", "everything", "tonight", "forever", "somebody's",
    "rock'n'roll", "1999", "2000", "Hallelujah", "OOH", "Yeah", "LOVE", "o'clock", "'til", "'cause",
};

static const char *SYL[] = {"ba", "be", "bi", "bo", "ca", "ce", "co", "da", "de", "di", "do", "fa",
                            "fe", "ga", "go", "ha", "he", "hi", "ja", "ka", "ki", "la", "le", "li",
                            "lo", "lu", "ma", "me", "mi", "mo", "na", "ne", "ni", "no", "pa", "pe",
                            "ra", "re", "ri", "ro", "sa", "se", "si", "so", "ta", "te", "ti", "to",
                            "va", "ve", "wa", "we", "ya", "yo", "za", "st", "tr", "ch", "sh", "th",
                            "ng", "er", "in", "on", "an", "ly", "ed", "es", "ous", "ight"};
#define NSYL (sizeof SYL / sizeof SYL[0])

/* Build word i of a generated vocabulary into buf (NUL terminated). */
static size_t vocab_word(uint32_t i, char *buf, int allow_long) {
    size_t nh = sizeof HEAD_WORDS / sizeof HEAD_WORDS[0];
    if (i < nh) {
        size_t l = strlen(HEAD_WORDS[i]);
        memcpy(buf, HEAD_WORDS[i], l + 1);
        return l;
    }
    Rng r = {0x5151000ULL + i * 0x9E37ULL};
    uint32_t nsyl = 1 + rng_below(&r, 4) + (rng_below(&r, 8) == 0 ? 2 : 0);
    if (allow_long && rng_below(&r, 64) == 0) nsyl += 6 + rng_below(&r, 8); /* 17..40 chars */
    size_t l = 0;
    for (uint32_t k = 0; k < nsyl; ++k) {
        const char *s = SYL[rng_below(&r, (uint32_t)NSYL)];
        size_t sl = strlen(s);
        memcpy(buf + l, s, sl);
        l += sl;
    }
    if (rng_below(&r, 11) == 0) buf[l++] = '\'';                /* rockin' */
    if (rng_below(&r, 13) == 0) buf[0] = (char)(buf[0] - 32);   /* Capitalised */
    if (rng_below(&r, 97) == 0) { buf[l++] = '0' + (char)(i % 10); }
    buf[l] = 0;
    return l;
}

static const char *ARTIST_PARTS[] = {"The", "Black", "Blue", "Silver", "Johnny", "Mary", "Kings", "of",
                                     "Leon", "Stone", "River", "Moon", "Sky", "Brothers", "Sisters",
                                     "Band", "Orchestra", "DJ", "Lil", "Big", "Ray", "Charles", "Elvis",
                                     "Presley", "Abba", "Queen", "Nirvana", "Bob", "Dylan", "Simon",
                                     "Garfunkel", "Earth", "Wind", "Fire", "Guns", "N'", "Roses",
                                     "Beyonc\xc3\xa9", "Sigur", "R\xc3\xb3s", "Mot\xc3\xb6rhead"};
#define NAP (sizeof ARTIST_PARTS / sizeof ARTIST_PARTS[0])

/* Artist j's display name; some contain ", " (then the field gets quoted),
 * some a '"' (escaped as "" inside the quoted field). */
static size_t artist_name(uint32_t j, char *buf, int *needs_quote) {
    Rng r = {0xA57157ULL + j * 0x2545F4914F6CDD1DULL};
    uint32_t parts = 1 + rng_below(&r, 3);
    size_t l = 0;
    *needs_quote = 0;
    for (uint32_t k = 0; k < parts; ++k) {
        const char *s = ARTIST_PARTS[rng_below(&r, (uint32_t)NAP)];
        size_t sl = strlen(s);
        if (k) {
            if (rng_below(&r, 9) == 0) { buf[l++] = ','; *needs_quote = 1; }
            buf[l++] = ' ';
        }
        memcpy(buf + l, s, sl);
        l += sl;
    }
    l += (size_t)(r.s & 0) ;
    /* make names distinct per j */
    l += (size_t)0;
    {
        char num[16];
        int nn = 0;
        uint32_t v = j;
        do { num[nn++] = (char)('0' + v % 10); v /= 10; } while (v);
        buf[l++] = ' ';
        while (nn) buf[l++] = num[--nn];
    }
    if (rng_below(&r, 50) == 0) {
        memcpy(buf + l, " \"The Kid\"", 10);
        l += 10;
        *needs_quote = 1;
    }
    buf[l] = 0;
    return l;
}

static void put_quoted(Out *o, const char *s, size_t n) {
    out_c(o, '"');
    for (size_t i = 0; i < n; ++i) {
        if (s[i] == '"') out_c(o, '"');
        out_c(o, s[i]);
    }
    out_c(o, '"');
}

/* The generation context shared (read-only) by every song: the rendered
 * vocabulary and the two Zipf samplers. */
typedef struct {
    const msa_gen_params *p;
    int highcard;
    uint32_t V, A, wps;
    Alias zw, za;
    char *arena;
    uint32_t *off;
} ZipfGen;

static int zipf_setup(ZipfGen *g, const msa_gen_params *p, int highcard) {
    memset(g, 0, sizeof *g);
    g->p = p;
    g->highcard = highcard;
    g->V = p->vocab ? p->vocab : 50000;
    g->A = p->n_artists ? p->n_artists : 5000;
    g->wps = p->words_per_song ? p->words_per_song : 30;
    if (alias_build(&g->zw, g->V, 1.0) || alias_build(&g->za, g->A, highcard ? 1.1 : 0.8)) return -1;
    g->arena = (char *)malloc((size_t)g->V * 48);
    g->off = (uint32_t *)malloc(sizeof(uint32_t) * (g->V + 1));
    if (!g->arena || !g->off) return -1;
    size_t al = 0;
    for (uint32_t i = 0; i < g->V; ++i) {
        g->off[i] = (uint32_t)al;
        al += vocab_word(i, g->arena + al, highcard);
    }
    g->off[g->V] = (uint32_t)al;
    return 0;
}
static void zipf_free(ZipfGen *g) {
    free(g->arena);
    free(g->off);
    alias_free(&g->zw);
    alias_free(&g->za);
}

/* Songs [s0, s1): each song draws from its own generator state (a function
 * of the seed and the song index), so any song range of the corpus can be
 * generated on its own -- a GPU's shard of a huge corpus, or a thread's. */
static void zipf_songs(const ZipfGen *g, uint64_t s0, uint64_t s1, Out *o) {
    const msa_gen_params *p = g->p;
    const int highcard = g->highcard;
    const uint32_t A = g->A, wps = g->wps;
    static const char *punct[] = {",", ".", "!", "?", " -", "...", ";", ":", ")", ""};
    char name[256], tmp[64];
    if (s0 == 0) {
        out_s(o, "artist,song,link,text");
        out_s(o, p->crlf ? "\r\n" : "\n");
    }
    for (uint64_t s = s0; s < s1; ++s) {
        Rng r = {p->seed * 0x9E3779B97F4A7C15ULL + 12345 + s * 0xD1342543DE82EF95ULL};
        (void)rng_next(&r);
        int q;
        /* highcard: half the songs by a skewed (Zipf 1.1) artist population,
         * half by one of 2^30 artists -> artist cardinality grows with songs */
        uint32_t aid = (highcard && rng_below(&r, 2)) ? A + rng_below(&r, 1u << 30) : alias_draw(&g->za, &r);
        size_t nl = artist_name(aid, name, &q);
        if (q) put_quoted(o, name, nl); else out_put(o, name, nl);
        out_c(o, ',');
        /* title: 1-4 vocab words, sometimes with a comma (quoted) */
        uint32_t tw = 1 + rng_below(&r, 4);
        int tq = rng_below(&r, 10) == 0;
        if (tq) out_c(o, '"');
        for (uint32_t k = 0; k < tw; ++k) {
            uint32_t w = alias_draw(&g->zw, &r);
            if (k) out_s(o, tq && k == 1 ? ", " : " ");
            out_put(o, g->arena + g->off[w], g->off[w + 1] - g->off[w]);
        }
        if (tq) out_c(o, '"');
        out_s(o, ",/a/");
        int n1 = 0;
        uint64_t v = s * 2654435761ULL % 100000000ULL;
        do { tmp[n1++] = (char)('0' + v % 10); v /= 10; } while (v);
        out_s(o, "song_");
        while (n1) out_c(o, tmp[--n1]);
        out_s(o, ".html,\"");
        /* lyrics: quoted, multi-line, escaped quotes now and then */
        uint32_t nw = wps / 2 + rng_below(&r, wps + 1);
        uint32_t line = 0;
        for (uint32_t k = 0; k < nw; ++k) {
            uint32_t w;
            if (highcard && rng_below(&r, 2) == 0) {
                /* unique-ish token: base-36 digits of random numbers, 60 % of
                 * them 3..8 bytes (S keys), 30 % 9..16 (M keys), 10 % 17..28
                 * (long words), so every table class sees high cardinality */
                const uint32_t cls = rng_below(&r, 10);
                const int want = cls < 6 ? 3 + (int)rng_below(&r, 6) : (cls < 9 ? 9 + (int)rng_below(&r, 8)
                                                                              : 17 + (int)rng_below(&r, 12));
                int t = 0;
                char tb[32];
                while (t < want) {
                    uint64_t x = rng_next(&r);
                    for (int d = 0; d < 12 && t < want; ++d) {
                        tb[t++] = "abcdefghijklmnopqrstuvwxyz0123456789"[x % 36];
                        x /= 36;
                    }
                }
                if (k && line) out_c(o, ' ');
                out_put(o, tb, (size_t)t);
                line++;
                continue;
            }
            w = alias_draw(&g->zw, &r);
            if (k && line) out_c(o, ' ');
            uint32_t deco = rng_below(&r, 64);
            if (deco == 0) out_s(o, "\"\"");
            else if (deco == 1) out_c(o, '(');
            out_put(o, g->arena + g->off[w], g->off[w + 1] - g->off[w]);
            if (deco == 0) out_s(o, "\"\"");
            else if (deco < 12) out_s(o, punct[deco % 10]);
            line++;
            if (line >= 5 + rng_below(&r, 5) && k + 1 < nw) {
                out_s(o, p->crlf ? "  \r\n" : "  \n");
                line = 0;
            }
        }
        out_s(o, "  \n\"");
        out_s(o, p->crlf ? "\r\n" : "\n");
    }
}

typedef struct {
    const ZipfGen *g;
    uint64_t s0, s1;
    Out o;
} GenJob;
static void *gen_job(void *arg) {
    GenJob *j = (GenJob *)arg;
    zipf_songs(j->g, j->s0, j->s1, &j->o);
    return NULL;
}

/* Songs [s0, s1) of the corpus, on up to 16 host threads for large ranges
 * (same bytes whatever the thread count). */
static void gen_zipf_like(const msa_gen_params *p, uint64_t s0, uint64_t s1, Out *o, int highcard) {
    ZipfGen g;
    if (zipf_setup(&g, p, highcard)) { o->oom = 1; zipf_free(&g); return; }
    const uint64_t n = s1 - s0;
    uint64_t nt = n / 200000;
    long ncpu = sysconf(_SC_NPROCESSORS_ONLN);
    if (nt > 16) nt = 16;
    if (ncpu > 0 && nt > (uint64_t)ncpu) nt = (uint64_t)ncpu;
    if (nt < 2) {
        zipf_songs(&g, s0, s1, o);
        zipf_free(&g);
        return;
    }
    GenJob jobs[16];
    pthread_t th[16];
    uint64_t started = 0;
    for (uint64_t t = 0; t < nt; ++t) {
        memset(&jobs[t].o, 0, sizeof(Out));
        jobs[t].g = &g;
        jobs[t].s0 = s0 + n * t / nt;
        jobs[t].s1 = s0 + n * (t + 1) / nt;
        if (t == 0 || pthread_create(&th[t], NULL, gen_job, &jobs[t]) != 0) {
            gen_job(&jobs[t]);  /* thread 0 (and any thread that failed to start) runs here */
            th[t] = 0;
        } else {
            started |= 1ull << t;
        }
    }
    for (uint64_t t = 1; t < nt; ++t)
        if (started >> t & 1ull) pthread_join(th[t], NULL);
    size_t tot = 0;
    for (uint64_t t = 0; t < nt; ++t) {
        if (jobs[t].o.oom) o->oom = 1;
        tot += jobs[t].o.n;
    }
    if (!o->oom) out_reserve(o, tot);
    for (uint64_t t = 0; t < nt; ++t) {
        if (!o->oom) {
            memcpy(o->p + o->n, jobs[t].o.p, jobs[t].o.n);
            o->n += jobs[t].o.n;
        }
        free(jobs[t].o.p);
    }
    zipf_free(&g);
}

/* CSV syntax torture: every state of the record reader, field splitter and
 * duplicate_field exercised, including NUL bytes and records with < 3 commas. */
static void gen_torture(const msa_gen_params *p, Out *o) {
    Rng r = {p->seed * 0xD1B54A32D192ED03ULL + 777};
    static const char *atoms[] = {"\"", "\"\"", ",", "\n", "\r", "\r\n", " ", "\t", "a", "Ab", "I'm",
                                  "don't", "xyz", "HELLO", "123", "''", "'", "word", "\xc3\xa9t\xc3\xa9",
                                  "\x00", "  ", "\"x\"", ",,", "\"a,b\"", "\f", "\v", "Z9'q"};
    static const size_t atom_len[] = {1, 2, 1, 1, 1, 2, 1, 1, 1, 2, 3, 5, 3, 5, 3, 2, 1, 4, 5, 1, 2, 3, 2, 5, 1, 1, 4};
    const uint32_t NA = (uint32_t)(sizeof atom_len / sizeof atom_len[0]);
    /* mostly well-formed header, sometimes odd */
    switch (rng_below(&r, 4)) {
    case 0: out_s(o, "artist,song,link,text\n"); break;
    case 1: out_s(o, " \"Art ist\" ,song,link, \"the text\" \r\n"); break;
    case 2: out_s(o, "artist,song,link,text"); out_s(o, "\r"); break;
    default: out_s(o, "a,b,c,\"multi\nline, header\"\n"); break;
    }
    for (uint64_t s = 0; s < p->n_songs; ++s) {
        uint32_t kind = rng_below(&r, 8);
        if (kind < 5) {
            /* plausible record with perturbed fields */
            uint32_t na = 1 + rng_below(&r, 4);
            int qa = rng_below(&r, 3) == 0;
            if (qa) out_c(o, '"');
            for (uint32_t k = 0; k < na; ++k) {
                uint32_t a = rng_below(&r, NA);
                if (qa || (atoms[a][0] != '"' && atoms[a][0] != ',' && atoms[a][0] != '\n' && atoms[a][0] != '\r'))
                    out_put(o, atoms[a], atom_len[a]);
                else
                    out_c(o, 'q');
            }
            if (qa) out_c(o, '"');
            out_s(o, rng_below(&r, 5) ? ",t," : ", \"t,1\" ,");
            out_s(o, "/l,");
            uint32_t nt = rng_below(&r, 24);
            int qt = rng_below(&r, 4) != 0;
            if (qt) out_s(o, rng_below(&r, 3) ? "\"" : "  \"");
            for (uint32_t k = 0; k < nt; ++k) {
                uint32_t a = rng_below(&r, NA);
                if (!qt && (atoms[a][0] == '\n' || atoms[a][0] == '\r')) { out_c(o, ' '); continue; }
                out_put(o, atoms[a], atom_len[a]);
            }
            if (qt) out_s(o, rng_below(&r, 3) ? "\"" : "\"  ");
            out_s(o, rng_below(&r, 6) ? "\n" : (rng_below(&r, 2) ? "\r\n" : "\r"));
        } else {
            /* raw atom soup: arbitrary parity, empty lines, short records */
            uint32_t n = rng_below(&r, 16);
            for (uint32_t k = 0; k < n; ++k) {
                uint32_t a = rng_below(&r, NA);
                out_put(o, atoms[a], atom_len[a]);
            }
            out_c(o, '\n');
        }
    }
}

int msa_gen_corpus_range(const msa_gen_params *p, uint64_t first_song, uint64_t n_songs, char **out, size_t *len) {
    if (!p || !out || !len) return -1;
    if (first_song > p->n_songs || n_songs > p->n_songs - first_song) return -1;
    if (p->mode == MSA_GEN_TORTURE && (first_song || n_songs != p->n_songs)) return -1;  /* one stream */
    Out o = {0};
    if (p->mode == MSA_GEN_TORTURE) gen_torture(p, &o);
    else gen_zipf_like(p, first_song, first_song + n_songs, &o, p->mode == MSA_GEN_HIGHCARD);
    if (o.oom) { free(o.p); return -2; }
    if (!o.p) { o.p = (char *)malloc(1); }
    *out = o.p;
    *len = o.n;
    return 0;
}

int msa_gen_corpus(const msa_gen_params *p, char **out, size_t *len) {
    if (!p) return -1;
    return msa_gen_corpus_range(p, 0, p->n_songs, out, len);
}

void msa_free(void *p) { free(p); }
