#!/usr/bin/env python3
"""Golden vectors for the column splitter (DESIGN.md row f, second script).

Runs the REAL reference script /root/reference/scripts/split_csv_columns.py
(in this container only) on deterministic inputs and stores, per case under
tests/golden/split/<case>/: input.csv, args.txt, the output files under out/
(names as the script chose them) and stdout.txt -- or error.txt when the
script exits non-zero.

    python tests/golden/make_split_golden.py
"""
import os
import random
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "split")
REF = "/root/reference/scripts/split_csv_columns.py"
sys.path.insert(0, HERE)


def cases():
    from make_wcs_golden import hand_cases, torture

    c = {}
    for k, (text, _) in hand_cases().items():
        c[k] = (text, ["--delimiter", ","])
    c["no_header"] = ("a,b,c\n1,2\n\n4,5,6,7\n", ["--delimiter", ",", "--no-header"])
    c["blank_first_no_header"] = ("\nx,y\n", ["--delimiter", ",", "--no-header"])
    c["dup_and_blank_headers"] = ("a b,a b,  ,A B,é/x\n1,2,3,4,5\n\"q,\"\"r\",\"\",x\ry,\"m\nn\",\n", ["--delimiter", ","])
    c["cr_values"] = ("h1,h2\n\"a\rb\",c\n", ["--delimiter", ","])
    for s in range(4):
        c[f"torture_{s}"] = (torture(500 + s, 120), ["--delimiter", ","])
    rnd = random.Random(9)
    rows = ["artist,song,link,text"]
    words = ["la", "love", "x,y", 'q""q', "nl\nnl"]
    for i in range(300):
        lyric = " ".join(rnd.choice(words) for _ in range(rnd.randint(0, 9)))
        rows.append("A%d,S%d,/l/%d,\"%s\"" % (rnd.randint(0, 40), i, i, lyric))
    c["lyrics_300"] = ("\n".join(rows) + "\n", ["--delimiter", ","])
    # no --delimiter: the script's detect_csv_params (csv.Sniffer) decides
    from make_wcs_golden import sniffed_cases

    for k, (text, _) in sniffed_cases().items():
        c[k] = (text, [])
    # sniffed skipinitialspace dialects (", " after every delimiter): spaces at
    # a field's start are dropped, a quote after them opens a quoted field
    c["sniff_skipinitialspace"] = ('a, b, c\n"x", "y", "z"\n"1", "2", "3"\n', [])
    c["sniff_skip_quoted_delims"] = ('h1, h2, h3\n1, "a, b", c\n2,   "x\ny", "q""q"\n3, , " lead"\n', [])
    c["sniff_skip_semicolon"] = ('name; value; note\nab; "c; d"; e\n  f;g ;  "h"\n', [])
    rows = ["artist, song, text"]
    for i in range(60):
        rows.append('A%d, S%d, "w%d, x %s"' % (i % 7, i, i, "y" * (i % 5)))
    c["sniff_skip_lyrics"] = ("\n".join(rows) + "\n", [])
    # --quotechar: the reader's and the writer's quote character
    q1 = ("artist,song,text\n'Art, ist',S1,'line one\nline \"two\"'\n"
          "B,'S''2',plain \"dq\" text\nC,it's,'a,b'\n'',x,'y'\n")
    c["quotechar_single"] = (q1, ["--delimiter", ",", "--quotechar", "'"])
    c["quotechar_single_sniffed"] = (q1.replace(",", ";"), ["--quotechar", "'"])
    c["quotechar_pipe"] = ("a,b\n|x,y|,|p||q|\n|multi\nline|,z\n", ["--delimiter", ",", "--quotechar", "|"])
    c["quotechar_dq_literal"] = ('a,b\n"x",y "z"\n', ["--delimiter", ",", "--quotechar", "'"])
    # --encoding utf-8: a BOM is the first header's first character (output
    # files without a BOM); utf-8-sig drops it and writes one per file
    bom = "\ufeff"
    c["utf8_bom"] = (bom + "artist,song\nA,\"x,y\"\n", ["--delimiter", ",", "--encoding", "utf-8"])
    c["utf8_no_bom"] = ("artist,song\nA,\"x,y\"\n", ["--delimiter", ",", "--encoding", "utf-8"])
    c["utf8_bom_sniffed"] = (bom + "a;b;c\n1;2;3\n4;\"5;6\";7\n", ["--encoding", "utf-8"])
    # single-byte codecs: every byte one character (the input written in that
    # codec; cases carry bytes)
    c["latin1_enc"] = ("artista,música,letra\nJosé,\"Ação, é\",\"olá\nmundo ü\"\nÁ,b,\"x\"\"y\"\n".encode("latin-1"),
                       ["--delimiter", ",", "--encoding", "latin-1"])
    c["latin1_sniffed"] = ("nome;cidade;nota\nJoão;São Paulo;ótimo\nÉlio;\"Brasília; DF\";bom\n".encode("latin-1"),
                           ["--encoding", "latin-1"])
    c["latin1_header_names"] = ("ção,ção,Ç ç,ÿ\n1,2,3,4\n5,6\n".encode("latin-1"),
                                ["--delimiter", ",", "--encoding", "iso-8859-1"])
    c["cp1252_enc"] = ("título,preço\n\"Café – 2€\",“aspas”\nx,ƒ\n".encode("cp1252"),
                       ["--delimiter", ",", "--encoding", "cp1252"])
    c["err_cp1252_undefined"] = (b"a,b\nx\x81y,z\n", ["--delimiter", ",", "--encoding", "cp1252"])
    return c


def main():
    if os.path.isdir(OUT):
        shutil.rmtree(OUT)
    os.makedirs(OUT)
    for name, (text, args) in sorted(cases().items()):
        d = os.path.join(OUT, name)
        os.makedirs(d)
        data = text if isinstance(text, bytes) else text.encode("utf-8")
        with open(os.path.join(d, "input.csv"), "wb") as f:
            f.write(data)
        with open(os.path.join(d, "args.txt"), "w") as f:
            f.write(" ".join(args))
        with tempfile.TemporaryDirectory() as tmp:
            od = os.path.join(tmp, "cols")
            r = subprocess.run([sys.executable, REF, os.path.join(d, "input.csv"), "--output-dir", od] + args,
                               capture_output=True, text=True)
            if r.returncode != 0:
                with open(os.path.join(d, "error.txt"), "w") as f:
                    f.write((r.stderr.strip().splitlines() or ["error"])[-1] + "\n")
                print(f"{name}: reference error: {(r.stderr.strip().splitlines() or ['?'])[-1]}")
                continue
            shutil.copytree(od, os.path.join(d, "out"))
            with open(os.path.join(d, "stdout.txt"), "w") as f:
                f.write(r.stdout.splitlines()[0].split(" arquivo")[0] + "\n")
            print(f"{name}: {sorted(os.listdir(od))}")


if __name__ == "__main__":
    main()
