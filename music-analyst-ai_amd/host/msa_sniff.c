/*
 * msa_sniff.c -- csv.Sniffer().sniff(sample) of CPython 3.10 (Lib/csv.py,
 * Sniffer.sniff / _guess_quote_and_delimiter / _guess_delimiter) restated in
 * C over the sample's code points.  Only what the two row (f) scripts read
 * from the dialect is produced: the delimiter and skipinitialspace.
 *
 * _guess_quote_and_delimiter's four regexes (DOTALL | MULTILINE, findall:
 * leftmost, non-overlapping, lazy ".*?") are matched directly: every
 * candidate start is tried in order, the lazy body takes the FIRST closing
 * that completes the pattern (found through per-(quote, delimiter) position
 * lists, so the whole sample costs O(n log n)).  \w is Python's Unicode word
 * class (str.isalnum() or '_', msa_unicode_word.h).  Dictionaries keep
 * insertion order and max() returns the first maximal key, as in Python.
 * tests/test_sniff.py compares this with the stdlib's csv.Sniffer.
 */
#include "msa_sniff.h"

#include <stdlib.h>
#include <string.h>

#include "msa_unicode_word.h"

long msa_sniff_sample(const unsigned char *b, size_t n, int utf8_sig, uint32_t *cps, size_t max_chars) {
    size_t i = 0, k = 0;
    if (utf8_sig && n >= 3 && b[0] == 0xEF && b[1] == 0xBB && b[2] == 0xBF) i = 3;  /* "utf-8" keeps U+FEFF */
    while (i < n && k < max_chars) {
        const uint32_t c = b[i];
        uint32_t cp, need, lo = 0x80, hi = 0xBF;
        if (c < 0x80) { cps[k++] = c; ++i; continue; }
        if (c < 0xC2) return -1;
        if (c < 0xE0) { need = 1; cp = c & 0x1F; }
        else if (c < 0xF0) { need = 2; cp = c & 0x0F; if (c == 0xE0) lo = 0xA0; if (c == 0xED) hi = 0x9F; }
        else if (c < 0xF5) { need = 3; cp = c & 0x07; if (c == 0xF0) lo = 0x90; if (c == 0xF4) hi = 0x8F; }
        else return -1;
        for (uint32_t j = 1; j <= need; ++j) {
            if (i + j >= n) return -1;
            const uint32_t d = b[i + j];
            if (j == 1 ? (d < lo || d > hi) : (d & 0xC0) != 0x80) return -1;
            cp = (cp << 6) | (d & 0x3F);
        }
        cps[k++] = cp;
        i += need + 1;
    }
    return (long)k;
}

static int is_word(uint32_t c) {
    if (c < 128) return (c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || c == '_';
    size_t lo = 0, hi = MSA_WORD_RANGES;
    while (lo < hi) {
        const size_t m = (lo + hi) / 2;
        if (c < msa_word_ranges[m][0]) hi = m;
        else if (c > msa_word_ranges[m][1]) lo = m + 1;
        else return 1;
    }
    return 0;
}
/* [^\w\n"'] */
static int is_dclass(uint32_t c) { return !is_word(c) && c != '\n' && c != '"' && c != '\''; }
static int is_quote(uint32_t c) { return c == '"' || c == '\''; }

/* insertion-ordered counter */
typedef struct {
    uint32_t *key;
    long *cnt;
    size_t n, cap;
} Counter;
static void ctr_add(Counter *c, uint32_t k) {
    for (size_t i = 0; i < c->n; ++i)
        if (c->key[i] == k) { ++c->cnt[i]; return; }
    if (c->n == c->cap) {
        c->cap = c->cap ? 2 * c->cap : 16;
        c->key = realloc(c->key, c->cap * sizeof *c->key);
        c->cnt = realloc(c->cnt, c->cap * sizeof *c->cnt);
    }
    c->key[c->n] = k;
    c->cnt[c->n++] = 1;
}
static size_t ctr_argmax(const Counter *c) {  /* first maximal key, as max(d, key=d.get) */
    size_t b = 0;
    for (size_t i = 1; i < c->n; ++i)
        if (c->cnt[i] > c->cnt[b]) b = i;
    return b;
}
static void ctr_free(Counter *c) { free(c->key); free(c->cnt); }

/* positions k with s[k] == q && s[k+1] == d, per (q, d) pair, built on demand */
typedef struct {
    uint32_t q, d;
    size_t *pos, n;
} PairList;
typedef struct {
    PairList *l;
    size_t n, cap;
} PairCache;
static const PairList *pairs_of(PairCache *pc, const uint32_t *s, size_t n, uint32_t q, uint32_t d) {
    for (size_t i = 0; i < pc->n; ++i)
        if (pc->l[i].q == q && pc->l[i].d == d) return &pc->l[i];
    if (pc->n == pc->cap) {
        pc->cap = pc->cap ? 2 * pc->cap : 8;
        pc->l = realloc(pc->l, pc->cap * sizeof *pc->l);
    }
    PairList *L = &pc->l[pc->n++];
    L->q = q;
    L->d = d;
    L->n = 0;
    L->pos = malloc((n ? n : 1) * sizeof *L->pos);
    for (size_t k = 0; k + 1 < n; ++k)
        if (s[k] == q && s[k + 1] == d) L->pos[L->n++] = k;
    return L;
}
static size_t first_at_or_after(const PairList *L, size_t p) {  /* SIZE_MAX: none */
    size_t lo = 0, hi = L->n;
    while (lo < hi) {
        const size_t m = (lo + hi) / 2;
        if (L->pos[m] < p) lo = m + 1;
        else hi = m;
    }
    return lo < L->n ? L->pos[lo] : (size_t)-1;
}

/* _guess_quote_and_delimiter: returns 1 with *delim / *skip when a delimiter
 * was found this way (else the caller runs _guess_delimiter) */
static int guess_quote_and_delimiter(const uint32_t *s, size_t n, uint32_t *delim, int *skip) {
    /* next_qd[qi][p]: smallest k >= p with s[k] == quote qi and s[k+1] in the delimiter class;
     * next_qe[qi][p]: ... and k + 1 == n or s[k+1] == '\n' */
    const uint32_t Q[2] = {'"', '\''};
    size_t *next_qd[2], *next_qe[2];
    for (int qi = 0; qi < 2; ++qi) {
        next_qd[qi] = malloc((n + 1) * sizeof(size_t));
        next_qe[qi] = malloc((n + 1) * sizeof(size_t));
        next_qd[qi][n] = next_qe[qi][n] = (size_t)-1;
        for (size_t k = n; k-- > 0;) {
            next_qd[qi][k] = (s[k] == Q[qi] && k + 1 < n && is_dclass(s[k + 1])) ? k : next_qd[qi][k + 1];
            next_qe[qi][k] = (s[k] == Q[qi] && (k + 1 == n || s[k + 1] == '\n')) ? k : next_qe[qi][k + 1];
        }
    }
    PairCache pc = {0};
    Counter quotes = {0}, delims = {0};
    long spaces = 0;
    int matched = 0, has_delim_group = 1;
    for (int pat = 1; pat <= 4 && !matched; ++pat) {
        has_delim_group = pat != 4;
        size_t i = 0;
        while (i < n) {
            size_t end = 0;
            uint32_t q = 0, d = 0;
            int sp = 0, ok = 0;
            if (pat == 1 || pat == 3) {
                /* (?P<delim>[^\w\n"'])(?P<space> ?)(?P<quote>["']).*?(?P=quote) then (?P=delim) | (?:$|\n) */
                if (is_dclass(s[i])) {
                    size_t j = i + 1;
                    if (j < n && s[j] == ' ') { sp = 1; ++j; }
                    if (j < n && is_quote(s[j])) {
                        q = s[j];
                        d = s[i];
                        size_t k;
                        if (pat == 1) k = first_at_or_after(pairs_of(&pc, s, n, q, d), j + 1);
                        else k = next_qe[q == '\''][j + 1];
                        if (k != (size_t)-1) {
                            ok = 1;
                            end = pat == 1 ? k + 2 : k + 1;
                        }
                    }
                }
            } else {
                /* (?:^|\n)(?P<quote>["']).*?(?P=quote) then (?P<delim>..)(?P<space> ?) | (?:$|\n) */
                for (int alt = 0; alt < 2 && !ok; ++alt) {
                    size_t qp;
                    if (alt == 0) {
                        if (!(i == 0 || s[i - 1] == '\n')) continue;
                        qp = i;
                    } else {
                        if (s[i] != '\n') continue;
                        qp = i + 1;
                    }
                    if (qp >= n || !is_quote(s[qp])) continue;
                    q = s[qp];
                    if (pat == 2) {
                        const size_t k = next_qd[q == '\''][qp + 1];
                        if (k == (size_t)-1) continue;
                        d = s[k + 1];
                        sp = (k + 2 < n && s[k + 2] == ' ');
                        end = k + 2 + (size_t)sp;
                    } else {
                        const size_t k = next_qe[q == '\''][qp + 1];
                        if (k == (size_t)-1) continue;
                        end = k + 1;
                    }
                    ok = 1;
                }
            }
            if (!ok) {
                ++i;
                continue;
            }
            matched = 1;
            ctr_add(&quotes, q);
            if (has_delim_group) {
                ctr_add(&delims, d);
                if (sp) ++spaces;
            }
            i = end;
        }
    }
    for (int qi = 0; qi < 2; ++qi) {
        free(next_qd[qi]);
        free(next_qe[qi]);
    }
    for (size_t i = 0; i < pc.n; ++i) free(pc.l[i].pos);
    free(pc.l);
    int found = 0;
    if (matched && delims.n) {
        const size_t b = ctr_argmax(&delims);
        if (delims.key[b] != '\n') {  /* always true: '\n' is not in the class */
            *delim = delims.key[b];
            *skip = delims.cnt[b] == spaces;
            found = 1;
        }
    }
    ctr_free(&quotes);
    ctr_free(&delims);
    return found;
}

/* str.count(sub) for sub = c or c + ' ' (non-overlapping) in [a, b) */
static long count1(const uint32_t *s, size_t a, size_t b, uint32_t c) {
    long r = 0;
    for (size_t i = a; i < b; ++i) r += s[i] == c;
    return r;
}
static long count2(const uint32_t *s, size_t a, size_t b, uint32_t c) {
    long r = 0;
    for (size_t i = a; i + 1 < b;) {
        if (s[i] == c && s[i + 1] == ' ') { ++r; i += 2; }
        else ++i;
    }
    return r;
}

typedef struct {
    long freq, cnt;
} FC;

/* _guess_delimiter */
static int guess_delimiter(const uint32_t *s, size_t n, uint32_t *delim, int *skip) {
    /* data = list(filter(None, data.split('\n'))) */
    size_t nl = 0, cap = 64;
    size_t *la = malloc(cap * sizeof *la), *lb = malloc(cap * sizeof *lb);
    for (size_t a = 0;;) {
        size_t b = a;
        while (b < n && s[b] != '\n') ++b;
        if (b > a) {
            if (nl == cap) {
                cap *= 2;
                la = realloc(la, cap * sizeof *la);
                lb = realloc(lb, cap * sizeof *lb);
            }
            la[nl] = a;
            lb[nl++] = b;
        }
        if (b >= n) break;
        a = b + 1;
    }
    const size_t chunk = nl < 10 ? nl : 10;
    /* charFrequency[c]: insertion-ordered (freq -> count) */
    FC *cf[127];
    size_t cfn[127], cfcap[127];
    for (int c = 0; c < 127; ++c) { cf[c] = NULL; cfn[c] = 0; cfcap[c] = 0; }
    /* modes, in insertion order */
    int mode_set[127] = {0}, mode_order[127], nmodes = 0;
    FC mode[127];
    /* delims, in insertion order */
    int dk[127], nd = 0;
    FC dv[127];
    int found = 0;
    size_t start = 0, end = chunk;
    long iteration = 0;
    while (start < nl) {
        ++iteration;
        for (size_t L = start; L < end && L < nl; ++L) {
            long h[127] = {0};
            for (size_t i = la[L]; i < lb[L]; ++i)
                if (s[i] < 127) ++h[s[i]];
            for (int c = 0; c < 127; ++c) {
                size_t j = 0;
                while (j < cfn[c] && cf[c][j].freq != h[c]) ++j;
                if (j == cfn[c]) {
                    if (cfn[c] == cfcap[c]) {
                        cfcap[c] = cfcap[c] ? 2 * cfcap[c] : 4;
                        cf[c] = realloc(cf[c], cfcap[c] * sizeof(FC));
                    }
                    cf[c][cfn[c]].freq = h[c];
                    cf[c][cfn[c]++].cnt = 0;
                }
                ++cf[c][j].cnt;
            }
        }
        for (int c = 0; c < 127; ++c) {
            if (cfn[c] == 1 && cf[c][0].freq == 0) continue;
            FC m;
            if (cfn[c] > 1) {
                size_t b = 0;
                for (size_t j = 1; j < cfn[c]; ++j)
                    if (cf[c][j].cnt > cf[c][b].cnt) b = j;
                long others = 0;
                for (size_t j = 0; j < cfn[c]; ++j)
                    if (j != b) others += cf[c][j].cnt;
                m.freq = cf[c][b].freq;
                m.cnt = cf[c][b].cnt - others;
            } else {
                m = cf[c][0];
            }
            if (!mode_set[c]) { mode_set[c] = 1; mode_order[nmodes++] = c; }
            mode[c] = m;
        }
        const size_t cl = chunk * (size_t)iteration;
        const double total = (double)(cl < nl ? cl : nl);
        double consistency = 1.0;
        const double threshold = 0.9;
        while (nd == 0 && consistency >= threshold) {
            for (int i = 0; i < nmodes; ++i) {
                const int c = mode_order[i];
                const FC v = mode[c];
                if (v.freq > 0 && v.cnt > 0 && ((double)v.cnt / total) >= consistency) {
                    int j = 0;
                    while (j < nd && dk[j] != c) ++j;
                    if (j == nd) dk[nd++] = c;
                    dv[j] = v;
                }
            }
            consistency -= 0.01;
        }
        if (nd == 1) {
            *delim = (uint32_t)dk[0];
            found = 1;
            break;
        }
        start = end;
        end += chunk;
    }
    if (!found && nd > 1) {
        static const uint32_t preferred[5] = {',', '\t', ';', ' ', ':'};
        for (int p = 0; p < 5 && !found; ++p)
            for (int j = 0; j < nd; ++j)
                if ((uint32_t)dk[j] == preferred[p]) { *delim = preferred[p]; found = 1; break; }
        if (!found) {  /* max of (v, k): freq, then adjusted count, then the character */
            int b = 0;
            for (int j = 1; j < nd; ++j) {
                const FC x = dv[j], y = dv[b];
                if (x.freq > y.freq || (x.freq == y.freq && (x.cnt > y.cnt || (x.cnt == y.cnt && dk[j] > dk[b])))) b = j;
            }
            *delim = (uint32_t)dk[b];
            found = 1;
        }
    }
    if (found) *skip = nl ? count1(s, la[0], lb[0], *delim) == count2(s, la[0], lb[0], *delim) : 0;
    for (int c = 0; c < 127; ++c) free(cf[c]);
    free(la);
    free(lb);
    return found;
}

msa_sniff_result msa_sniff(const uint32_t *s, size_t n) {
    msa_sniff_result r = {0, 0, 0};
    uint32_t d = 0;
    int skip = 0;
    if (guess_quote_and_delimiter(s, n, &d, &skip) || guess_delimiter(s, n, &d, &skip)) {
        r.ok = 1;
        r.delimiter = d;
        r.skipinitialspace = skip;
    }
    return r;
}
