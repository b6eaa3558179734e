/*
 * msa_sniff_test -- prints what the C csv.Sniffer restatement (msa_sniff.c)
 * decides for each file given: "<ok> <delimiter code point> <skipinitialspace>"
 * per line, or "decode-error".  tests/test_sniff.py compares the output with
 * the stdlib's csv.Sniffer on the same samples.
 */
#include <stdio.h>
#include <stdlib.h>

#include "msa_sniff.h"

int main(int argc, char **argv) {
    for (int a = 1; a < argc; ++a) {
        FILE *f = fopen(argv[a], "rb");
        if (!f) { printf("open-error\n"); continue; }
        size_t cap = 1 << 20, n = 0;
        unsigned char *b = malloc(cap);
        for (size_t got; (got = fread(b + n, 1, cap - n, f)) > 0;) {
            n += got;
            if (n == cap) b = realloc(b, cap *= 2);
        }
        fclose(f);
        uint32_t *cps = malloc(65536 * sizeof *cps);
        const long k = msa_sniff_sample(b, n, 1, cps, 65536);
        if (k < 0) printf("decode-error\n");
        else {
            const msa_sniff_result r = msa_sniff(cps, (size_t)k);
            printf("%d %u %d\n", r.ok, r.ok ? r.delimiter : 0u, r.ok ? r.skipinitialspace : 0);
        }
        free(cps);
        free(b);
    }
    return 0;
}
