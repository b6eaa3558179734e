"""CPU: which --encoding values the column splitter's byte path takes
(msa.single_byte_codec, msa/split_columns.py).  The GPU splitter works on
bytes; that is the script's answer exactly when every byte decodes to at most
one character, bytes below 0x80 to themselves, and decode + encode is the
identity -- so the per-column bytes it writes are the input's bytes.  This
pins the classification against Python's own codecs (the ones
split_csv_columns.py:130,179 open the files with)."""
import codecs
import random

import pytest


@pytest.mark.parametrize("enc", ["latin-1", "iso-8859-1", "iso-8859-15", "cp1252", "cp1250", "cp437", "koi8-r",
                                 "mac-roman", "ascii", "windows-1252", "latin_1"])
def test_single_byte_codecs_accepted(enc):
    from msa import single_byte_codec

    bad = single_byte_codec(enc)
    assert bad is not None
    name = codecs.lookup(enc).name
    for b in range(256):
        raw = bytes([b])
        if b in bad:
            with pytest.raises(UnicodeDecodeError):
                raw.decode(name)
            continue
        ch = raw.decode(name)
        assert len(ch) == 1 and ch.encode(name) == raw
        if b < 0x80:
            assert ch == chr(b)


@pytest.mark.parametrize("enc", ["utf-8", "utf-8-sig", "utf-16", "utf-32", "shift_jis", "gbk", "big5", "euc-kr",
                                 "euc-jp", "no-such-codec"])
def test_other_codecs_refused(enc):
    from msa import single_byte_codec

    assert single_byte_codec(enc) is None


@pytest.mark.parametrize("enc", ["latin-1", "cp1252", "koi8-r"])
def test_byte_path_is_the_identity(enc):
    """Random text in the codec: decoding and encoding back gives the same
    bytes, so a byte-level split writes what the script writes."""
    from msa import single_byte_codec

    bad = single_byte_codec(enc)
    ok = [b for b in range(1, 256) if b not in bad]
    rnd = random.Random(7)
    data = bytes(rnd.choice(ok) for _ in range(20000))
    assert data.decode(enc).encode(enc) == data
