/*
 * msa_sniff.h -- csv.Sniffer().sniff(sample) (CPython 3.10 Lib/csv.py) in C,
 * for the C host of the row (f) scripts:
 *   word_count_per_song.py detect_delimiter (42-49): the sniffed delimiter,
 *     ',' when sniff raises;
 *   split_csv_columns.py detect_csv_params (48-66): delimiter and
 *     skipinitialspace, ',' / False when sniff raises.
 * The sample is the script's fh.read(65536): the first 65536 characters of
 * the file decoded as UTF-8 ("utf-8-sig": a leading BOM is not part of it).
 */
#ifndef MSA_SNIFF_H
#define MSA_SNIFF_H

#include <stddef.h>
#include <stdint.h>

typedef struct {
    int ok;                /* 0: sniff raised csv.Error ("Could not determine delimiter") */
    uint32_t delimiter;    /* code point */
    int skipinitialspace;
} msa_sniff_result;

/* Decode the script's sample from the raw file bytes: skip a UTF-8 BOM when
 * utf8_sig ("utf-8-sig"; "utf-8" keeps it as U+FEFF), take up to max_chars
 * code points.  Returns the number of code points written to
 * cps (capacity max_chars), or -1 when the bytes are not valid UTF-8 within
 * the sample (the script's read() raises UnicodeDecodeError). */
long msa_sniff_sample(const unsigned char *bytes, size_t n, int utf8_sig, uint32_t *cps, size_t max_chars);

msa_sniff_result msa_sniff(const uint32_t *s, size_t n);

#endif
