#!/usr/bin/env python3
"""Golden vectors for the per-song word counter (SURVEY §8 row f).

Runs the REAL reference script /root/reference/scripts/word_count_per_song.py
(in this container only) on deterministic inputs and stores input + outputs
under tests/golden/wcs/<case>/:
    input.csv, args.txt, word_counts_by_song.csv, word_counts_global.csv,
    rows.txt (the "Processadas N linhas" count) -- or error.txt when the
    reference exits non-zero (the GPU path must refuse the same inputs).

    python tests/golden/make_wcs_golden.py
"""
import os
import random
import re
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
# inputs WITHOUT --delimiter (args.txt empty) exercise the script's csv.Sniffer
OUT = os.path.join(HERE, "wcs")
REF = "/root/reference/scripts/word_count_per_song.py"
sys.path.insert(0, os.path.join(HERE, "..", "..", "music-analyst-ai_amd"))

HDR = "artist,song,link,text\n"


def hand_cases():
    c = {}
    c["basic"] = (HDR + 'ABBA,Song One,/a/1,"Hello hello HELLO world, it\'s the world"\n'
                  'Queen,Two,/a/2,"We will rock you\nwe WILL rock"\n'), []
    c["latin1_letters"] = (HDR + 'Édith Piaf,Non,/x,"ÀÉÎÕÜ àéîõü ßßß ÞÞÞ þþþ aa×bb ÷÷÷ Ça ÇAVA çava ÿÿÿ ŸŸŸ naïve NAÏVE"\n'
                           'B,C,/y,"Ærøskøbing ÆRØSKØBING øøø ØØØ 123 4567 a1b"\n'), []
    c["apostrophes"] = (HDR + "A,S,/l,\"''' '' 'a' ''b ab' don't DON'T o'clock ''''' x''\"\n"), ["--delimiter", ","]
    c["quotes"] = (HDR + 'A,S,/l,"say ""hello"" now ""quoted""" \n'
                   '"Art, ist","So""ng",/l,"ab"cd efg"hij, and more"\n'
                   'Plain,Song,/l,unquoted words here "with quote" inside\n'), ["--delimiter", ","]
    c["crlf_cr_blank"] = ("artist,song,link,text\r\n\r\nA,S1,/l,\"line one\r\nline two\rline three\"\r\n\r\n"
                          "B,S2,/l,plain text words\r\r\nC,S3,/l,\"last one without newline\""), ["--delimiter", ","]
    c["bom_and_strip"] = ("﻿" + HDR + "  A  , Song　,/l,\"words words words\"\n"
                          " B ,\tS\t,/l,\"more words\"\n \x1cC\x1f , S ,/l,\"\u0085zzz\u0085\"\n"), ["--delimiter", ","]
    c["col_order_dupes"] = ("text,x,song,artist,text\nignored,1,S1,A1,\"real text here\"\n"
                            "other,2,S2,A2,second text body,extra,fields\n"), ["--delimiter", ","]
    c["empty_texts"] = (HDR + 'A,S,/l,""\nB,T,/l,"a b c"\nC,U,/l,"to go"\nD,V,/l,"yes"\n'), ["--delimiter", ","]
    c["unterminated"] = (HDR + 'A,S,/l,"never closed words\nkeep going, more words\n'), ["--delimiter", ","]
    c["short_row_ok"] = ("artist,song,text,link\nA,S,some text words\nB,T,more text words,/l\n"), ["--delimiter", ","]
    c["err_short_row"] = (HDR + "A,S\n"), ["--delimiter", ","]
    c["err_missing_col"] = ("artist,title,link,text\nA,S,/l,words\n"), ["--delimiter", ","]
    c["err_blank_first"] = ("\n" + HDR + "A,S,/l,words\n"), ["--delimiter", ","]
    c["header_only"] = (HDR), ["--delimiter", ","]
    c["quoted_header"] = ('"artist","song",link,"te\nxt"\n"A",S,/l,x\n'
                          '"artist","song",link,text\nB,T,/l,"header as data words"\n'), ["--delimiter", ","]
    c["whitespace_only"] = (HDR + '   ,   ,/l,"word word"\n　, ,/l,"other"\n'), ["--delimiter", ","]
    return c


def torture(seed, n):
    rnd = random.Random(seed)
    alpha = ["a", "b", "Z", "q", "é", "É", "ß", "'", "1", " ", ",", '"', '""', "\n", "\r\n", "\r", "-", "×",
             "ÿ", "Ω", "中", " ", "the", "THE", "Love", "don't", "naïve", "x"]
    out = ["artist,song,link,text\n"]
    for _ in range(n):
        def fld(q):
            s = "".join(rnd.choice(alpha) for _ in range(rnd.randint(0, 12)))
            if q:
                return '"' + s.replace('"', '""') + '"' + (rnd.choice(["", "", "", "x", " y"]))
            return s.replace(",", " ").replace("\n", " ").replace("\r", " ").replace('"', "'")
        row = [fld(rnd.random() < 0.5) for _ in range(3)]
        txt = fld(True) if rnd.random() < 0.8 else fld(False)
        out.append(",".join(row) + "," + txt + rnd.choice(["\n", "\r\n", "\n\n", "\r"]))
    return "".join(out)


def zipf(n, seed, crlf=False):
    import msa

    return msa.gen_corpus(n, mode="zipf", seed=seed, crlf=crlf).decode("utf-8")


def sniffed_cases():
    """Inputs run WITHOUT --delimiter: the script's detect_delimiter (csv.Sniffer
    on the first 65536 characters) picks the delimiter."""
    rnd = random.Random(77)
    words = ["love", "the", "naïve", "don't", "you", "Über", "night", "ÇA", "x", "rock'n'roll"]

    def lyric(d):
        body = " ".join(rnd.choice(words) for _ in range(rnd.randint(1, 12)))
        if rnd.random() < 0.5:
            body = body.replace(" ", d + " ", 1) + ", yeah"
        return '"' + body.replace('"', '""') + '\n' + rnd.choice(words) + '"'

    c = {}
    for name, d in (("sniff_semicolon", ";"), ("sniff_tab", "\t"), ("sniff_pipe", "|"), ("sniff_colon", ":")):
        rows = [d.join(["artist", "song", "link", "text"])]
        for i in range(60):
            rows.append(d.join([f"Artist {i % 7}", f"Song {i}", f"/l/{i}", lyric(d)]))
        c[name] = ("\n".join(rows) + "\n", [])
    # unquoted, space separated: the frequency heuristic (_guess_delimiter) decides
    c["sniff_space_unquoted"] = ("artist song text\n" + "".join(f"A{i} S{i} word{i % 5}\n" for i in range(40)), [])
    # no quotes, no consistent character: sniff raises, ',' is used
    c["sniff_fails"] = ("artist,song,link,text\nA,S,/l,some words here, and more\nB,T\n"
                        "C,U,/l,x,y,z,w,v\nsingle\n", [])
    # the generated lyric corpus with ';' (the shape of the real dataset)
    import msa

    z = msa.gen_corpus(150, mode="zipf", seed=5).decode("utf-8")
    out, q = [], False
    for ch in z:  # ',' -> ';' outside quotes
        if ch == '"':
            q = not q
        out.append(";" if (ch == "," and not q) else ch)
    c["sniff_zipf_semicolon"] = ("".join(out), [])
    return c


def main():
    cases = hand_cases()
    cases.update(sniffed_cases())
    for s in range(6):
        cases[f"torture_{s}"] = (torture(100 + s, 150), ["--delimiter", ","])
    # --encoding utf-8: a BOM is not stripped -- it becomes the first header
    # name's first character (the required "artist" column is then missing
    # when it is the first column) and is part of the Sniffer's sample
    bom = "\ufeff"
    cases["utf8_bom_artist_first"] = (bom + HDR + 'A,S,/l,"hello there world"\n', ["--encoding", "utf-8"])
    cases["utf8_bom_id_first"] = (bom + "id,artist,song,text\n1,A,S,\"hello there world\"\n2,B,T,\"more words here\"\n",
                                  ["--encoding", "utf-8"])
    cases["utf8_bom_sniffed"] = (bom + "id;artist;song;text\n1;A;S;\"hello; there world\"\n2;B;T;more words here\n",
                                 ["--encoding", "utf-8"])
    cases["utf8_no_bom"] = (HDR + 'A,S,/l,"hello there, world"\nB,T,/m,words words words\n', ["--encoding", "utf-8"])
    cases["utf8_sig_explicit"] = (bom + HDR + 'A,S,/l,"hello there, world"\n', ["--encoding", "utf-8-sig"])
    cases["zipf_300"] = (zipf(300, 3), [])
    cases["zipf_crlf_200"] = (zipf(200, 7, crlf=True), [])
    if os.path.isdir(OUT):
        shutil.rmtree(OUT)
    os.makedirs(OUT)
    for name, (text, args) in sorted(cases.items()):
        d = os.path.join(OUT, name)
        os.makedirs(d)
        data = text.encode("utf-8")
        with open(os.path.join(d, "input.csv"), "wb") as f:
            f.write(data)
        with open(os.path.join(d, "args.txt"), "w") as f:
            f.write(" ".join(args))
        with tempfile.TemporaryDirectory() as tmp:
            r = subprocess.run([sys.executable, REF, os.path.join(d, "input.csv"), "--output-dir", tmp, "--workers", "1"]
                               + args, capture_output=True, text=True)
            if r.returncode != 0:
                with open(os.path.join(d, "error.txt"), "w") as f:
                    f.write((r.stderr.strip().splitlines() or ["error"])[-1] + "\n")
                print(f"{name}: reference error: {(r.stderr.strip().splitlines() or ['?'])[-1]}")
                continue
            m = re.search(r"Processadas (\d+) linhas", r.stdout)
            with open(os.path.join(d, "rows.txt"), "w") as f:
                f.write(m.group(1) + "\n")
            for fn in ("word_counts_by_song.csv", "word_counts_global.csv"):
                shutil.copy(os.path.join(tmp, fn), os.path.join(d, fn))
            print(f"{name}: {m.group(1)} rows")


if __name__ == "__main__":
    main()
