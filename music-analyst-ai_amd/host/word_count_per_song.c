/*
 * word_count_per_song -- drop-in CLI for /root/reference/scripts/
 * word_count_per_song.py (main 102-155) on libmsa_hip's GPU path (msa_wcs_*).
 *
 *   word_count_per_song <csv> [--output-dir D] [--delimiter C]
 *                       [--encoding utf-8-sig] [--workers N]
 *
 * Writes D/word_counts_global.csv and D/word_counts_by_song.csv (default D =
 * output/serial_word_counts) and prints the script's three lines.  --workers
 * is accepted and ignored (the GPU replaces the thread pool, 132-133).
 * Without --delimiter the delimiter is detect_delimiter's (42-49):
 * csv.Sniffer on the first 65536 characters, ',' when it fails (msa_sniff.c
 * restates the stdlib's Sniffer).  The GPU reader takes any one-byte ASCII
 * delimiter but '"', CR, LF; a sniffed or given delimiter outside that set,
 * and encodings other than UTF-8, are refused.  --encoding utf-8 keeps a BOM
 * as data (U+FEFF in the first header name, as the script's DictReader sees
 * it); utf-8-sig, the default, drops it.
 */
#define _POSIX_C_SOURCE 200809L
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include "msa_hip.h"
#include "msa_sniff.h"

static int mkdirs(const char *path) {
    char tmp[4096];
    size_t n = strlen(path);
    if (n == 0 || n >= sizeof tmp) return -1;
    memcpy(tmp, path, n + 1);
    for (size_t i = 1; i <= n; ++i) {
        if (tmp[i] == '/' || tmp[i] == 0) {
            char c = tmp[i];
            tmp[i] = 0;
            if (mkdir(tmp, 0777) != 0 && errno != EEXIST) return -1;
            tmp[i] = c;
        }
    }
    return 0;
}

static char *read_file(const char *path, size_t *len) {
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    size_t cap = 1 << 20, n = 0;
    char *b = malloc(cap);
    for (;;) {
        if (n == cap) {
            cap *= 2;
            b = realloc(b, cap);
        }
        size_t k = fread(b + n, 1, cap - n, f);
        n += k;
        if (k == 0) break;
    }
    fclose(f);
    *len = n;
    return b;
}

/* os.fspath(Path(p)) (POSIX pathlib): repeated slashes and "." components
 * collapse, a trailing slash goes, ".." stays, exactly two leading slashes
 * are kept, "" becomes "." -- the script prints its paths this way (148-155). */
static void path_norm(const char *p, char *out, size_t cap) {
    size_t o = 0;
    const size_t n = strlen(p);
    if (n >= 2 && p[0] == '/' && p[1] == '/' && (n == 2 || p[2] != '/')) { out[o++] = '/'; out[o++] = '/'; }
    else if (n >= 1 && p[0] == '/') out[o++] = '/';
    const size_t root = o;
    for (size_t i = 0; i < n;) {
        while (i < n && p[i] == '/') ++i;
        size_t j = i;
        while (j < n && p[j] != '/') ++j;
        const size_t len = j - i;
        if (len && !(len == 1 && p[i] == '.') && o + len + 2 < cap) {
            if (o > root) out[o++] = '/';
            memcpy(out + o, p + i, len);
            o += len;
        }
        i = j;
    }
    if (o == 0) out[o++] = '.';
    out[o] = 0;
}

int main(int argc, char **argv) {
    const char *csv = NULL, *outdir = "output/serial_word_counts", *delim = NULL, *enc = "utf-8-sig";
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--output-dir") && i + 1 < argc) outdir = argv[++i];
        else if (!strcmp(argv[i], "--delimiter") && i + 1 < argc) delim = argv[++i];
        else if (!strcmp(argv[i], "--encoding") && i + 1 < argc) enc = argv[++i];
        else if (!strcmp(argv[i], "--workers") && i + 1 < argc) ++i;
        else if (!csv) csv = argv[i];
        else {
            fprintf(stderr, "usage: %s <csv> [--output-dir D] [--delimiter C] [--encoding utf-8-sig]\n", argv[0]);
            return 2;
        }
    }
    if (!csv) {
        fprintf(stderr, "usage: %s <csv> [--output-dir D] [--delimiter C] [--encoding utf-8-sig]\n", argv[0]);
        return 2;
    }
    if (delim && strlen(delim) != 1) {
        /* csv.DictReader(delimiter=...) raises TypeError: "delimiter" must be a 1-character string */
        fprintf(stderr, "TypeError: \"delimiter\" must be a 1-character string\n");
        return 1;
    }
    if (strcmp(enc, "utf-8-sig") != 0 && strcmp(enc, "utf-8") != 0 && strcmp(enc, "utf8") != 0) {
        fprintf(stderr, "only UTF-8 input is implemented on the GPU path\n");
        return 2;
    }
    struct stat st;
    if (stat(csv, &st) != 0) {
        fprintf(stderr, "Arquivo não encontrado: %s\n", csv);
        return 1;
    }
    if (mkdirs(outdir) != 0) {
        fprintf(stderr, "cannot create %s\n", outdir);
        return 1;
    }
    size_t n = 0;
    char *data = read_file(csv, &n);
    if (!data) {
        fprintf(stderr, "cannot read %s\n", csv);
        return 1;
    }
    /* "utf-8" (not "utf-8-sig") keeps a BOM: U+FEFF is the sample's first
     * character and the first header name's first character (main 111-115) */
    const int utf8_sig = strcmp(enc, "utf-8-sig") == 0;
    uint32_t dch = delim ? (unsigned char)delim[0] : ',';
    if (!delim) {  /* detect_delimiter(fh.read(65536)) */
        uint32_t *cps = malloc(65536 * sizeof *cps);
        const long k = msa_sniff_sample((const unsigned char *)data, n, utf8_sig, cps, 65536);
        if (k < 0) {
            fprintf(stderr, "UnicodeDecodeError: 'utf-8' codec can't decode the first 65536 characters of %s\n", csv);
            free(cps);
            free(data);
            return 1;
        }
        const msa_sniff_result sr = msa_sniff(cps, (size_t)k);
        free(cps);
        dch = sr.ok ? sr.delimiter : ',';
    }
    if (dch == 0 || dch > 127 || dch == '"' || dch == '\r' || dch == '\n') {
        fprintf(stderr, "delimiter U+%04X is not implemented on the GPU path\n", (unsigned)dch);
        free(data);
        return 2;
    }
    msa_wcs *w = NULL;
    int rc = msa_wcs_create(0, &w);
    if (rc) {
        fprintf(stderr, "msa_wcs_create failed (%d): no GPU visible\n", rc);
        return 1;
    }
    rc = msa_wcs_set_delimiter(w, (int)dch);
    if (!rc) rc = msa_wcs_set_encoding(w, utf8_sig);
    if (!rc) rc = msa_wcs_load_csv(w, data, n);
    free(data);
    if (!rc) rc = msa_wcs_run(w);
    if (!rc) rc = msa_wcs_write_outputs(w, outdir);
    if (rc) {
        fprintf(stderr, "%s\n", msa_wcs_last_error(w));
        msa_wcs_destroy(w);
        return 1;
    }
    msa_wcs_summary s;
    msa_wcs_get_summary(w, &s);
    msa_wcs_destroy(w);
    char shown[4096];
    path_norm(outdir, shown, sizeof shown);
    const char *sep = strcmp(shown, "/") && strcmp(shown, "//") ? "/" : "";
    printf("Concluído. Processadas %llu linhas. Arquivos gerados em %s\n", (unsigned long long)s.total_rows, shown);
    if (!strcmp(shown, ".")) {  /* Path(".") / "x" is "x" */
        printf(" - word_counts_global.csv\n");
        printf(" - word_counts_by_song.csv\n");
    } else {
        printf(" - %s%sword_counts_global.csv\n", shown, sep);
        printf(" - %s%sword_counts_by_song.csv\n", shown, sep);
    }
    return 0;
}
