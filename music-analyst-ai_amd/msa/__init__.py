"""ctypes binding of libmsa_hip (include/msa_hip.h) for tests, bench.py and smoke().

The product is C: libmsa_hip.so (gfx950 HIP kernels behind a C ABI) and the
drop-in CLI bin/parallel_spotify (music-analyst-ai_amd/host/parallel_spotify.c,
mirroring /root/reference/src/parallel_spotify.c:724-1113).  This module only
drives that library from Python.  There is no fallback: if libmsa_hip.so is
missing, or no GPU is visible, every call raises.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("MSA_LIB") or os.path.join(PKG_DIR, "libmsa_hip.so")
CLI_PATH = os.path.join(PKG_DIR, "bin", "parallel_spotify")
GEN_PATH = os.path.join(PKG_DIR, "bin", "msa_gen")

MSA_OK = 0
MSA_ERR = {
    -1: "MSA_ERR_ARG",
    -2: "MSA_ERR_HIP",
    -3: "MSA_ERR_NOHEADER",
    -4: "MSA_ERR_BADHEADER",
    -5: "MSA_ERR_CAPACITY",
    -6: "MSA_ERR_COLLISION",
    -7: "MSA_ERR_IO",
    -8: "MSA_ERR_INPUT",
}
MSA_SPLIT_TEXT_COLUMN = 1
MSA_TABLE_WORDS = 0
MSA_TABLE_ARTISTS = 1
GEN_MODES = {"zipf": 0, "highcard": 1, "torture": 2}
PROF_MAX = 16

# Every symbol include/msa_hip.h declares (tests check the .so exports them).
EXPORTS = [
    "msa_gen_corpus", "msa_gen_corpus_range", "msa_free", "msa_build_id", "msa_create", "msa_destroy", "msa_last_error",
    "msa_stream", "msa_sync", "msa_load_csv", "msa_bind_csv", "msa_split_columns",
    "msa_count", "msa_rank", "msa_run", "msa_get_summary", "msa_get_ranked",
    "msa_write_table_csv", "msa_get_split_column", "msa_set_profiling", "msa_get_profile",
    "msa_set_shard", "msa_piece_size", "msa_shard_function", "msa_shard_head", "msa_segment_copy",
    "msa_segment_set", "msa_artist_reader_needed", "msa_set_artist_reader", "msa_export_partitions", "msa_export_ranked", "msa_export_copy", "msa_import_partitions", "msa_import_ranked",
    "msa_wcs_create", "msa_wcs_destroy", "msa_wcs_last_error", "msa_wcs_stream", "msa_wcs_load_csv",
    "msa_wcs_set_table_bits", "msa_wcs_set_delimiter", "msa_wcs_set_quoting", "msa_wcs_set_dialect", "msa_wcs_set_encoding", "msa_wcs_run", "msa_wcs_get_summary", "msa_wcs_get_csv", "msa_wcs_write_outputs",
    "msa_csvcol_run", "msa_csvcol_header", "msa_csvcol_get",
]
MSA_WCS_GLOBAL = 0
MSA_WCS_BY_SONG = 1
PIECE_CSV = 0
PIECE_ARTISTS = 1
SHARD_FN_BYTES = 120  # sizeof(msa_shard_fn)


def single_byte_codec(encoding: str):
    """For an ASCII-compatible single-byte codec (every byte decodes to at most
    one character, bytes < 0x80 to themselves, and decode + encode is the
    identity on the bytes it defines): the bytes it leaves undefined (a
    frozenset, empty for latin-1).  None for any other codec (UTF-8, UTF-16,
    multi-byte Asian codecs, unknown names)."""
    import codecs

    try:
        info = codecs.lookup(encoding)
    except LookupError:
        return None
    if info.name in ("utf-8", "utf-8-sig"):
        return None
    bad = set()
    for b in range(256):
        try:
            ch = bytes([b]).decode(info.name)
        except UnicodeDecodeError:
            bad.add(b)
            continue
        except Exception:
            return None
        if len(ch) != 1 or (b < 0x80 and ch != chr(b)):
            return None
        try:
            if ch.encode(info.name) != bytes([b]):
                return None
        except Exception:
            return None
    if any(b < 0x80 for b in bad):
        return None
    for b in bad:  # a byte that only fails alone is a multi-byte lead (Shift-JIS, GBK, ...)
        for x in range(0x40, 0x100):
            try:
                bytes([b, x]).decode(info.name)
                return None
            except UnicodeDecodeError:
                pass
    return frozenset(bad)


class MsaError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{MSA_ERR.get(code, code)}: {msg}")
        self.code = code


class _GenParams(C.Structure):
    _fields_ = [
        ("seed", C.c_uint64),
        ("n_songs", C.c_uint64),
        ("vocab", C.c_uint32),
        ("n_artists", C.c_uint32),
        ("words_per_song", C.c_uint32),
        ("mode", C.c_int),
        ("crlf", C.c_int),
    ]


class _Summary(C.Structure):
    _fields_ = [
        ("total_songs", C.c_longlong),
        ("total_words", C.c_longlong),
        ("n_words", C.c_uint64),
        ("n_artists", C.c_uint64),
        ("n_records", C.c_uint64),
        ("artist_label", C.c_char * 128),
        ("text_label", C.c_char * 128),
        ("artist_file", C.c_char * 128),
        ("text_file", C.c_char * 128),
    ]


class _Profile(C.Structure):
    _fields_ = [
        ("n", C.c_int),
        ("name", (C.c_char * 32) * PROF_MAX),
        ("ms", C.c_double * PROF_MAX),
        ("launches", C.c_uint64 * PROF_MAX),
        ("bytes", C.c_uint64 * PROF_MAX),
    ]


class _WcsSummary(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("total_rows", "song_rows", "total_tokens", "n_words", "n_pairs",
                                                   "fallback_rows")]


_lib = None


def load(path: str = LIB_PATH):
    """Load libmsa_hip.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} not built: run `make -C music-analyst-ai_amd` (or __graft_entry__.build())")
    lib = C.CDLL(path)
    vp, sz, u64, i = C.c_void_p, C.c_size_t, C.c_uint64, C.c_int
    lib.msa_gen_corpus.argtypes = [C.POINTER(_GenParams), C.POINTER(C.c_void_p), C.POINTER(sz)]
    lib.msa_gen_corpus_range.argtypes = [C.POINTER(_GenParams), u64, u64, C.POINTER(C.c_void_p), C.POINTER(sz)]
    lib.msa_free.argtypes = [vp]
    lib.msa_free.restype = None
    lib.msa_build_id.argtypes = []
    lib.msa_build_id.restype = C.c_char_p
    lib.msa_create.argtypes = [i, C.POINTER(vp)]
    lib.msa_destroy.argtypes = [vp]
    lib.msa_destroy.restype = None
    lib.msa_last_error.argtypes = [vp]
    lib.msa_last_error.restype = C.c_char_p
    lib.msa_stream.argtypes = [vp]
    lib.msa_stream.restype = vp
    lib.msa_sync.argtypes = [vp]
    lib.msa_load_csv.argtypes = [vp, vp, sz]
    lib.msa_bind_csv.argtypes = [vp, vp, sz]
    lib.msa_split_columns.argtypes = [vp, i]
    lib.msa_count.argtypes = [vp]
    lib.msa_rank.argtypes = [vp]
    lib.msa_run.argtypes = [vp, i]
    lib.msa_get_summary.argtypes = [vp, C.POINTER(_Summary)]
    lib.msa_get_ranked.argtypes = [vp, i, u64, u64, C.POINTER(C.c_longlong), C.POINTER(u64), C.c_char_p, u64,
                                   C.POINTER(u64)]
    lib.msa_write_table_csv.argtypes = [vp, i, C.c_char_p, C.c_char_p, i]
    lib.msa_get_split_column.argtypes = [vp, i, C.POINTER(C.c_void_p), C.POINTER(sz)]
    lib.msa_set_shard.argtypes = [vp, i]
    lib.msa_piece_size.argtypes = [vp, i, C.POINTER(u64)]
    lib.msa_shard_function.argtypes = [vp, i, vp]
    lib.msa_shard_head.argtypes = [vp, i, vp, i, C.POINTER(u64), C.POINTER(u64)]
    lib.msa_segment_copy.argtypes = [vp, i, u64, u64, vp]
    lib.msa_segment_set.argtypes = [vp, i, u64, vp, u64]
    lib.msa_artist_reader_needed.argtypes = [vp, C.POINTER(i)]
    lib.msa_set_artist_reader.argtypes = [vp, i]
    lib.msa_export_partitions.argtypes = [vp, i, i, C.POINTER(u64)]
    lib.msa_export_copy.argtypes = [vp, vp]
    lib.msa_export_ranked.argtypes = [vp, i, u64, C.POINTER(u64)]
    lib.msa_import_partitions.argtypes = [vp, i, vp, C.POINTER(u64), i]
    lib.msa_import_ranked.argtypes = [vp, i, vp, C.POINTER(u64), i]
    lib.msa_set_profiling.argtypes = [vp, i]
    lib.msa_get_profile.argtypes = [vp, C.POINTER(_Profile), i]
    lib.msa_wcs_create.argtypes = [i, C.POINTER(vp)]
    lib.msa_wcs_destroy.argtypes = [vp]
    lib.msa_wcs_destroy.restype = None
    lib.msa_wcs_last_error.argtypes = [vp]
    lib.msa_wcs_last_error.restype = C.c_char_p
    lib.msa_wcs_stream.argtypes = [vp]
    lib.msa_wcs_stream.restype = vp
    lib.msa_wcs_load_csv.argtypes = [vp, vp, sz]
    lib.msa_wcs_set_table_bits.argtypes = [vp, i]
    lib.msa_wcs_set_delimiter.argtypes = [vp, i]
    lib.msa_wcs_set_quoting.argtypes = [vp, i, i]
    lib.msa_wcs_set_dialect.argtypes = [vp, i, i, i]
    lib.msa_wcs_set_encoding.argtypes = [vp, i]
    lib.msa_wcs_run.argtypes = [vp]
    lib.msa_wcs_get_summary.argtypes = [vp, C.POINTER(_WcsSummary)]
    lib.msa_wcs_get_csv.argtypes = [vp, i, C.POINTER(C.c_void_p), C.POINTER(sz)]
    lib.msa_wcs_write_outputs.argtypes = [vp, C.c_char_p]
    lib.msa_csvcol_run.argtypes = [vp, i, C.POINTER(u64), C.POINTER(u64)]
    lib.msa_csvcol_header.argtypes = [vp, u64, C.POINTER(C.c_void_p), C.POINTER(sz)]
    lib.msa_csvcol_get.argtypes = [vp, u64, C.POINTER(C.c_void_p), C.POINTER(sz)]
    _lib = lib
    return lib


def build_id() -> str:
    """msa_build_id(): hash of the sources + flags this libmsa_hip.so was built from."""
    return load().msa_build_id().decode()


def _bytes_at(ptr, n: int) -> bytes:
    """bytes of a malloc'ed C buffer (ctypes.string_at truncates sizes to 32 bits)."""
    if n == 0:
        return b""
    return bytes((C.c_ubyte * n).from_address(ptr.value if isinstance(ptr, C.c_void_p) else ptr))


def gen_corpus(n_songs: int, mode: str = "zipf", seed: int = 1, vocab: int = 50000, n_artists: int = 5000,
               words_per_song: int = 30, crlf: bool = False, first_song: int = 0,
               count: Optional[int] = None) -> bytes:
    """Deterministic synthetic corpus (csrc/msa_gen.c) -- host code, no GPU.
    With first_song / count: only songs [first_song, first_song + count) of the
    n_songs-song corpus (header only in the range starting at song 0)."""
    lib = load()
    p = _GenParams(seed, n_songs, vocab, n_artists, words_per_song, GEN_MODES[mode], int(crlf))
    out = C.c_void_p()
    n = C.c_size_t()
    if count is None and first_song == 0:
        rc = lib.msa_gen_corpus(C.byref(p), C.byref(out), C.byref(n))
    else:
        cnt = n_songs - first_song if count is None else count
        rc = lib.msa_gen_corpus_range(C.byref(p), first_song, cnt, C.byref(out), C.byref(n))
    if rc:
        raise MsaError(rc, "corpus generation failed")
    try:
        return _bytes_at(out, n.value)
    finally:
        lib.msa_free(out)


@dataclass
class Summary:
    total_songs: int
    total_words: int
    n_words: int
    n_artists: int
    n_records: int
    artist_label: bytes
    text_label: bytes
    artist_file: str
    text_file: str


class Context:
    """One msa_ctx: one GPU, one HIP stream (msa_create / msa_destroy)."""

    def __init__(self, device: int = 0):
        self.lib = load()
        h = C.c_void_p()
        rc = self.lib.msa_create(device, C.byref(h))
        if rc:
            raise MsaError(rc, f"msa_create(device={device}) failed (no GPU visible?)")
        self.h = h

    def close(self):
        if self.h:
            self.lib.msa_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc: int):
        if rc:
            raise MsaError(rc, (self.lib.msa_last_error(self.h) or b"").decode(errors="replace"))

    @property
    def stream(self) -> int:
        return self.lib.msa_stream(self.h) or 0

    def load_csv(self, data: bytes):
        self._check(self.lib.msa_load_csv(self.h, data, len(data)))

    def bind_csv(self, dev_ptr: int, n: int):
        self._check(self.lib.msa_bind_csv(self.h, C.c_void_p(dev_ptr), n))

    def split_columns(self, text_column: bool = True):
        self._check(self.lib.msa_split_columns(self.h, MSA_SPLIT_TEXT_COLUMN if text_column else 0))

    def count(self):
        self._check(self.lib.msa_count(self.h))

    def rank(self):
        self._check(self.lib.msa_rank(self.h))

    def run(self, text_column: bool = True):
        self._check(self.lib.msa_run(self.h, MSA_SPLIT_TEXT_COLUMN if text_column else 0))

    def sync(self):
        self._check(self.lib.msa_sync(self.h))

    def set_profiling(self, on: bool = True):
        self._check(self.lib.msa_set_profiling(self.h, int(on)))

    def profile(self, reset: bool = False) -> Dict[str, dict]:
        """HIP-event time per pipeline stage, accumulated since the last reset."""
        p = _Profile()
        self._check(self.lib.msa_get_profile(self.h, C.byref(p), int(reset)))
        out = {}
        for k in range(p.n):
            out[p.name[k].value.decode()] = {"ms": p.ms[k], "launches": p.launches[k], "bytes": p.bytes[k]}
        return out

    # ---- multi-GPU shard API (msa/dist.py drives it)
    def set_shard(self, first: bool):
        self._check(self.lib.msa_set_shard(self.h, int(first)))

    def piece_size(self, piece: int) -> int:
        v = C.c_uint64()
        self._check(self.lib.msa_piece_size(self.h, piece, C.byref(v)))
        return v.value

    def shard_function(self, piece: int) -> bytes:
        buf = C.create_string_buffer(SHARD_FN_BYTES)
        self._check(self.lib.msa_shard_function(self.h, piece, buf))
        return buf.raw

    def shard_head(self, piece: int, fns_before: List[bytes], sizes_before: List[int]) -> int:
        k = len(fns_before)
        blob = C.create_string_buffer(b"".join(fns_before), max(1, SHARD_FN_BYTES * k))
        sizes = (C.c_uint64 * max(1, k))(*sizes_before)
        v = C.c_uint64()
        self._check(self.lib.msa_shard_head(self.h, piece, blob, k, sizes, C.byref(v)))
        return v.value

    def segment_copy(self, piece: int, off: int, length: int, dst_ptr: int):
        self._check(self.lib.msa_segment_copy(self.h, piece, off, length, C.c_void_p(dst_ptr)))

    def segment_set(self, piece: int, skip: int, tail_ptr: int = 0, tail_len: int = 0):
        self._check(self.lib.msa_segment_set(self.h, piece, skip, C.c_void_p(tail_ptr or None), tail_len))

    def artist_reader_needed(self) -> bool:
        v = C.c_int()
        self._check(self.lib.msa_artist_reader_needed(self.h, C.byref(v)))
        return bool(v.value)

    def set_artist_reader(self, exact: bool):
        self._check(self.lib.msa_set_artist_reader(self.h, int(exact)))

    def export_partitions(self, table: int, nparts: int) -> List[int]:
        out = (C.c_uint64 * nparts)()
        self._check(self.lib.msa_export_partitions(self.h, table, nparts, out))
        return list(out)

    def export_ranked(self, table: int, limit: int = 0) -> int:
        """Serialise ranked entries [0, limit) (all: 0) as one wire block; returns its bytes."""
        n = C.c_uint64()
        self._check(self.lib.msa_export_ranked(self.h, table, limit, C.byref(n)))
        return n.value

    def export_copy(self, dst_ptr: int):
        self._check(self.lib.msa_export_copy(self.h, C.c_void_p(dst_ptr)))

    def import_partitions(self, table: int, src_ptr: int, blk_off: List[int]):
        arr = (C.c_uint64 * len(blk_off))(*blk_off)
        self._check(self.lib.msa_import_partitions(self.h, table, C.c_void_p(src_ptr or None), arr, len(blk_off) - 1))

    def import_ranked(self, table: int, src_ptr: int, blk_off: List[int]):
        """Root of the final gather: merge the GPUs' ranked blocks (msa_import_ranked)."""
        arr = (C.c_uint64 * len(blk_off))(*blk_off)
        self._check(self.lib.msa_import_ranked(self.h, table, C.c_void_p(src_ptr or None), arr, len(blk_off) - 1))

    def summary(self) -> Summary:
        s = _Summary()
        self._check(self.lib.msa_get_summary(self.h, C.byref(s)))
        return Summary(s.total_songs, s.total_words, s.n_words, s.n_artists, s.n_records, s.artist_label,
                       s.text_label, s.artist_file.decode(), s.text_file.decode())

    def ranked(self, table: int, first: int = 0, count: Optional[int] = None) -> List[Tuple[bytes, int]]:
        s = self.summary()
        n = s.n_words if table == MSA_TABLE_WORDS else s.n_artists
        if count is None:
            count = max(0, n - first)
        count = min(count, max(0, n - first))
        need = C.c_uint64()
        self._check(self.lib.msa_get_ranked(self.h, table, first, count, None, None, None, 0, C.byref(need)))
        counts = (C.c_longlong * max(count, 1))()
        offs = (C.c_uint64 * (count + 1))()
        keys = C.create_string_buffer(need.value + 1)
        self._check(self.lib.msa_get_ranked(self.h, table, first, count, counts, offs, keys, need.value + 1,
                                            C.byref(need)))
        raw = keys.raw
        return [(raw[offs[i]:offs[i + 1]], counts[i]) for i in range(count)]

    def write_table_csv(self, table: int, path: str, key_header: str, limit: int = 0):
        self._check(self.lib.msa_write_table_csv(self.h, table, path.encode(), key_header.encode(), limit))

    def split_column(self, which: int) -> bytes:
        out = C.c_void_p()
        n = C.c_size_t()
        self._check(self.lib.msa_get_split_column(self.h, which, C.byref(out), C.byref(n)))
        try:
            return _bytes_at(out, n.value)
        finally:
            self.lib.msa_free(out)


def table_csv_bytes(entries: List[Tuple[bytes, int]], key_header: str, limit: int = 0) -> bytes:
    """write_table_csv's byte format (parallel_spotify.c:307-344) for a ranked list."""
    if limit > 0:
        entries = entries[:limit]
    out = [key_header.encode() + b",count\n"]
    for k, c in entries:
        out.append(b'"' + k.replace(b'"', b'""') + b'",' + str(c).encode() + b"\n")
    return b"".join(out)


class WordCountPerSong:
    """Per-song word counter on the GPU (msa_wcs_*): the drop-in for
    /root/reference/scripts/word_count_per_song.py's counting.  ``run(data)``
    returns (rows processed, word_counts_by_song.csv bytes,
    word_counts_global.csv bytes) -- the values the script prints/writes."""

    def __init__(self, device: int = 0):
        self.lib = load()
        h = C.c_void_p()
        rc = self.lib.msa_wcs_create(device, C.byref(h))
        if rc:
            raise MsaError(rc, f"msa_wcs_create(device={device}) failed (no GPU visible?)")
        self.h = h

    def close(self):
        if self.h:
            self.lib.msa_wcs_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc: int):
        if rc:
            raise MsaError(rc, (self.lib.msa_wcs_last_error(self.h) or b"").decode(errors="replace"))

    @property
    def stream(self) -> int:
        return self.lib.msa_wcs_stream(self.h) or 0

    def load_csv(self, data: bytes):
        self._check(self.lib.msa_wcs_load_csv(self.h, data, len(data)))

    def set_table_bits(self, bits: int):
        self._check(self.lib.msa_wcs_set_table_bits(self.h, bits))

    def set_delimiter(self, delimiter: str):
        """The reader's field delimiter (one ASCII character, not the quotechar, CR, LF or NUL)."""
        if len(delimiter) != 1:
            raise MsaError(-1, f"delimiter must be one character, got {delimiter!r}")
        self._check(self.lib.msa_wcs_set_delimiter(self.h, ord(delimiter)))

    def set_quoting(self, quotechar: str = '"', skipinitialspace: bool = False):
        """The column splitter's quotechar and skipinitialspace (split_csv_columns.py)."""
        if len(quotechar) != 1:
            raise MsaError(-1, f"quotechar must be one character, got {quotechar!r}")
        self._check(self.lib.msa_wcs_set_quoting(self.h, ord(quotechar), 1 if skipinitialspace else 0))

    def set_dialect(self, delimiter: str, quotechar: str = '"', skipinitialspace: bool = False):
        """Delimiter + quotechar + skipinitialspace at once, validated as a pair (msa_wcs_set_dialect)."""
        if len(delimiter) != 1 or len(quotechar) != 1:
            raise MsaError(-1, f"delimiter/quotechar must be one character, got {delimiter!r}/{quotechar!r}")
        self._check(self.lib.msa_wcs_set_dialect(self.h, ord(delimiter), ord(quotechar), 1 if skipinitialspace else 0))

    def set_encoding(self, encoding: str = "utf-8-sig"):
        """--encoding: "utf-8-sig" drops a leading BOM, "utf-8" keeps it as data;
        a single-byte ASCII-compatible codec (latin-1, cp1252, ...: see
        single_byte_codec) reads every byte as one character (the column
        splitter only)."""
        e = encoding.lower().replace("_", "-")
        if e in ("utf-8-sig", "utf-8", "utf8"):
            self._check(self.lib.msa_wcs_set_encoding(self.h, 1 if e == "utf-8-sig" else 0))
        elif single_byte_codec(encoding) is not None:
            self._check(self.lib.msa_wcs_set_encoding(self.h, 2))
        else:
            raise MsaError(-1, f"only UTF-8 and single-byte ASCII-compatible encodings are implemented, not {encoding!r}")

    def count(self):
        self._check(self.lib.msa_wcs_run(self.h))

    def summary(self) -> dict:
        s = _WcsSummary()
        self._check(self.lib.msa_wcs_get_summary(self.h, C.byref(s)))
        return {n: getattr(s, n) for n, _ in _WcsSummary._fields_}

    def csv(self, which: int) -> bytes:
        out = C.c_void_p()
        n = C.c_size_t()
        self._check(self.lib.msa_wcs_get_csv(self.h, which, C.byref(out), C.byref(n)))
        try:
            return _bytes_at(out, n.value)
        finally:
            self.lib.msa_free(out)

    def write_outputs(self, outdir: str):
        self._check(self.lib.msa_wcs_write_outputs(self.h, outdir.encode()))

    # ---- column splitter (split_csv_columns.py), same context
    def split_columns(self, has_header: bool = True) -> Tuple[int, int]:
        nc, nr = C.c_uint64(), C.c_uint64()
        self._check(self.lib.msa_csvcol_run(self.h, int(has_header), C.byref(nc), C.byref(nr)))
        return nc.value, nr.value

    def _take(self, fn, col: int) -> bytes:
        out = C.c_void_p()
        n = C.c_size_t()
        self._check(fn(self.h, col, C.byref(out), C.byref(n)))
        try:
            return _bytes_at(out, n.value)
        finally:
            self.lib.msa_free(out)

    def column_header(self, col: int) -> bytes:
        return self._take(self.lib.msa_csvcol_header, col)

    def column_body(self, col: int) -> bytes:
        return self._take(self.lib.msa_csvcol_get, col)

    def run(self, data: bytes) -> Tuple[int, bytes, bytes]:
        self.load_csv(data)
        self.count()
        return self.summary()["total_rows"], self.csv(MSA_WCS_BY_SONG), self.csv(MSA_WCS_GLOBAL)
