/*
 * msa_gen -- write a deterministic synthetic corpus (see csrc/msa_gen.c).
 *
 *   msa_gen <out.csv> [--songs N] [--seed S] [--vocab V] [--artists A]
 *           [--words W] [--mode zipf|highcard|torture] [--crlf]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "msa_hip.h"

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s <out.csv> [--songs N] [--seed S] [--vocab V] [--artists A] [--words W] "
                        "[--mode zipf|highcard|torture] [--crlf]\n", argv[0]);
        return 1;
    }
    msa_gen_params p = {1, 1000, 50000, 5000, 30, MSA_GEN_ZIPF, 0};
    for (int i = 2; i < argc; ++i) {
        if (!strcmp(argv[i], "--songs") && i + 1 < argc) p.n_songs = strtoull(argv[++i], 0, 10);
        else if (!strcmp(argv[i], "--seed") && i + 1 < argc) p.seed = strtoull(argv[++i], 0, 10);
        else if (!strcmp(argv[i], "--vocab") && i + 1 < argc) p.vocab = (uint32_t)atoi(argv[++i]);
        else if (!strcmp(argv[i], "--artists") && i + 1 < argc) p.n_artists = (uint32_t)atoi(argv[++i]);
        else if (!strcmp(argv[i], "--words") && i + 1 < argc) p.words_per_song = (uint32_t)atoi(argv[++i]);
        else if (!strcmp(argv[i], "--crlf")) p.crlf = 1;
        else if (!strcmp(argv[i], "--mode") && i + 1 < argc) {
            const char *m = argv[++i];
            p.mode = !strcmp(m, "highcard") ? MSA_GEN_HIGHCARD : !strcmp(m, "torture") ? MSA_GEN_TORTURE : MSA_GEN_ZIPF;
        } else {
            fprintf(stderr, "unknown argument %s\n", argv[i]);
            return 1;
        }
    }
    char *buf = NULL;
    size_t n = 0;
    if (msa_gen_corpus(&p, &buf, &n)) { fprintf(stderr, "generation failed\n"); return 1; }
    FILE *fp = fopen(argv[1], "wb");
    if (!fp || fwrite(buf, 1, n, fp) != n) { fprintf(stderr, "cannot write %s\n", argv[1]); return 1; }
    fclose(fp);
    msa_free(buf);
    printf("%zu\n", n);
    return 0;
}
