"""Debug helper: run the GPU per-song counter on tiny inputs and print outputs."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "music-analyst-ai_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import msa  # noqa: E402
import wcs_oracle  # noqa: E402

cases = [b"artist,song,link,text\nA,S,/l,abc def\n", b"artist,song,link,text\nA,S,/l,\"abc def abc\"\nB,T,/l,xyz\n"]
with msa.WordCountPerSong(0) as w:
    for d in cases:
        print(repr(d))
        print(" gpu   ", w.run(d), w.summary())
        print(" oracle", wcs_oracle.word_count_per_song(d))
