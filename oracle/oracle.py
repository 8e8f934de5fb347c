"""ORACLE / TEST INFRASTRUCTURE ONLY -- never imported by the product path.

Python face of the CPU restatement in ``oracle/ambc_oracle.c`` plus the parts
of the reference that are easiest to restate in Python:

* ``decompress_body`` -- ``AdaptiveCompressor._adaptive_decompress``
  (adaptive_compressor.py:396-454) including every lenient path, with the C
  per-codec decoders and stdlib zlib/bz2/lzma for ids 5/6/7
  (advanced_compression.py:83-96,124-137,187-200), and id 8 (zstandard,
  :236-250) restated over the system libzstd -- parity unpinned: the reference
  holds no zstd fixture and python-zstandard is absent.
* ``compress_file_bytes`` -- ``AdaptiveCompressor.compress``
  (adaptive_compressor.py:221-255) around the C body loop, with the reference's
  stats dicts (:457-532).
* ``entropy_table`` -- numpy's ``p * np.log2(p)`` per count, the exact terms
  ``HuffmanCompression.should_use`` sums (compression_methods.py:566-571).

Pinned by tests/test_oracle.py against tests/golden/ (vectors produced by the
reference itself, see tests/golden/make_golden.py).
"""
import bz2
import ctypes as C
import hashlib
import lzma
import os
import struct
import subprocess
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libambc_oracle.so")
MARKER = b"\xff\xff\x00\x00"

# adaptive_compressor.py:114-127
PREFS = {1: (32, 4096), 2: (128, 8192), 3: (32, 8192), 4: (32, 4096), 5: (64, 65536),
         6: (1024, 262144), 7: (8192, 524288), 8: (512, 262144), 9: (1024, 65536),
         10: (1024, 262144), 11: (1024, 262144), 255: (1, 999999999)}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH) and os.path.exists("/usr/bin/make"):
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        _lib = C.CDLL(LIB_PATH)
        u8p, i64, u32 = C.c_void_p, C.c_int64, C.c_uint32
        for name in ("orc_rle_encode", "orc_huff_encode", "orc_dict_encode",
                     "orc_lz4_frame_encode", "orc_lz4_block_encode", "orc_deflate_encode",
                     "orc_gd_encode"):
            getattr(_lib, name).argtypes = [u8p, u32, u8p]
            getattr(_lib, name).restype = i64
        for name in ("orc_rle_decode", "orc_huff_decode", "orc_delta_decode", "orc_dict_decode",
                     "orc_lz4_frame_decode"):
            getattr(_lib, name).argtypes = [u8p, u32, u32, u8p]
            getattr(_lib, name).restype = i64
        for name in ("orc_rle_should_use", "orc_delta_should_use", "orc_dict_should_use",
                     "orc_deflate_should_use"):
            getattr(_lib, name).argtypes = [u8p, u32]
            getattr(_lib, name).restype = C.c_int
        _lib.orc_huff_should_use.argtypes = [u8p, u32, u8p]
        _lib.orc_dict_encode_wl.argtypes = [u8p, u32, C.c_int64, C.c_int64, u8p]
        _lib.orc_dict_encode_wl.restype = i64
        _lib.orc_gd_parse.argtypes = [u8p, u32, u8p]
        _lib.orc_gd_parse.restype = u32
        _lib.orc_huff_should_use.restype = C.c_int
        _lib.orc_huff_entropy.argtypes = [u8p, u32, u8p]
        _lib.orc_huff_entropy.restype = C.c_double
        _lib.orc_huff_code_table.argtypes = [C.c_int, u8p, u8p, u8p, u8p]
        _lib.orc_huff_code_table.restype = C.c_int
        _lib.orc_xxh32.argtypes = [u8p, C.c_uint64, C.c_uint32]
        _lib.orc_xxh32.restype = C.c_uint32
        _lib.orc_synth.argtypes = [u8p, C.c_uint64, C.c_uint64]
        _lib.orc_random_bytes.argtypes = [u8p, C.c_uint64, C.c_uint64]
        _lib.orc_select.argtypes = [u8p, u32, C.c_void_p, u8p, C.POINTER(C.c_int64)]
        _lib.orc_select.restype = C.c_int
        _lib.orc_decide_all.argtypes = [u8p, C.c_uint64, C.c_void_p, u8p, u8p, C.c_int]
        _lib.orc_compress_body.argtypes = [u8p, C.c_uint64, C.c_void_p, u8p, C.c_uint64,
                                           C.c_void_p, C.c_int]
        _lib.orc_compress_body.restype = i64
    return _lib


class Params(C.Structure):
    _fields_ = [("chunk_size", C.c_uint32), ("mode", C.c_uint32), ("method_mask", C.c_uint32),
                ("flags", C.c_uint32), ("pref_min", C.c_uint32 * 16),
                ("pref_max", C.c_uint32 * 16), ("ent_full", C.c_void_p),
                ("ent_tail", C.c_void_p)]


class Stats(C.Structure):
    _fields_ = [("method_usage", C.c_uint64 * 256), ("total_chunks", C.c_uint64),
                ("compressed_chunks", C.c_uint64), ("raw_chunks", C.c_uint64),
                ("bytes_saved", C.c_uint64), ("payload_bytes", C.c_uint64),
                ("overhead_bytes", C.c_uint64)]


def _buf(data):
    b = (C.c_uint8 * max(1, len(data))).from_buffer_copy(bytes(data) or b"\0")
    return b


def entropy_table(n):
    """numpy's term p*np.log2(p) for p = c/n, c = 0..n (c=0 unused)."""
    c = np.arange(n + 1, dtype=np.float64)
    p = c / float(n)
    with np.errstate(divide="ignore", invalid="ignore"):
        t = p * np.log2(p)
    t[0] = 0.0
    return np.ascontiguousarray(t)


def _call_enc(fn, data, bound):
    L = lib()
    src = _buf(data)
    out = (C.c_uint8 * max(1, bound))()
    r = getattr(L, fn)(C.addressof(src), len(data), C.addressof(out))
    return None if r < 0 else bytes(out[:r])


def rle_encode(d):
    return _call_enc("orc_rle_encode", d, 2 * len(d) + 2)


def huff_encode(d):
    return _call_enc("orc_huff_encode", d, 1 + 5 * 256 + 4 + 8 * len(d) + 8)


def dict_encode(d):
    return _call_enc("orc_dict_encode", d, 2 * len(d) + 4)


def dict_encode_wl(d, window_size, lookahead_size):
    """DictionaryCompression(window_size, lookahead_size).compress(d) for any
    window, lookahead and length (orc_dict_encode_wl); ValueError where the
    reference's bytearray.append raises (a match longer than 255 bytes)."""
    L = lib()
    src = _buf(d)
    out = (C.c_uint8 * max(1, 2 * len(d) + 4))()
    clamp = lambda v: max(-(1 << 62), min(1 << 62, int(v)))
    r = L.orc_dict_encode_wl(C.addressof(src), len(d), clamp(window_size), clamp(lookahead_size),
                             C.addressof(out))
    if r == -2:
        raise ValueError("byte must be in range(0, 256)")
    return bytes(out[:r])


def lz4_frame_encode(d):
    return _call_enc("orc_lz4_frame_encode", d, len(d) + len(d) // 255 + 64)


def deflate_encode(d):
    """zlib.compress(d, level=9) through the same system zlib CPython links."""
    return _call_enc("orc_deflate_encode", d, len(d) + len(d) // 1000 + 64)


def gdeflate_encode(d):
    """"ambc-deflate v1" (the GPU engine's id-5 encoder) -> zlib stream."""
    return _call_enc("orc_gd_encode", d, len(d) + 5 * (len(d) // 65535 + 1) + 64)


def gd_parse(d):
    """"ambc-deflate v1" greedy parse -> list of (pos, length, distance)."""
    L = lib()
    src = _buf(d)
    out = (C.c_uint32 * (3 * (len(d) // 4 + 2)))()
    ns = L.orc_gd_parse(C.addressof(src), len(d), C.addressof(out))
    return [tuple(out[3 * i:3 * i + 3]) for i in range(ns)]


def lz4_block_encode(d):
    return _call_enc("orc_lz4_block_encode", d, len(d) + len(d) // 255 + 64)


def should_use(mid, d, tab=None):
    L, src = lib(), _buf(d)
    if mid == 1:
        return bool(L.orc_rle_should_use(C.addressof(src), len(d)))
    if mid == 2:
        return bool(L.orc_dict_should_use(C.addressof(src), len(d)))
    if mid == 4:
        return bool(L.orc_delta_should_use(C.addressof(src), len(d)))
    if mid == 5:
        return bool(L.orc_deflate_should_use(C.addressof(src), len(d)))
    if mid == 3:
        t = entropy_table(len(d)) if (tab is None and len(d) > 0) else tab
        return bool(L.orc_huff_should_use(C.addressof(src), len(d),
                                          t.ctypes.data if t is not None else None))
    raise ValueError(mid)


def huff_entropy(d, tab=None):
    src = _buf(d)
    return lib().orc_huff_entropy(C.addressof(src), len(d),
                                  tab.ctypes.data if tab is not None else None)


def huff_code_table(hist):
    """hist: list of (symbol, weight) in table order -> {sym: code-string}."""
    k = len(hist)
    syms = (C.c_uint8 * 256)(*[s for s, _ in hist])
    ws = (C.c_uint64 * 256)(*[w for _, w in hist])
    lens = (C.c_uint8 * 256)()
    codes = (C.c_uint64 * 256)()
    if lib().orc_huff_code_table(k, C.addressof(syms), C.addressof(ws), C.addressof(lens),
                                 C.addressof(codes)):
        return None
    return {s: format(codes[s], "0%db" % lens[s]) if lens[s] else "" for s, _ in hist}


def xxh32(b, seed=0):
    src = _buf(b)
    return lib().orc_xxh32(C.addressof(src), len(b), seed)


def synth(n, seed=20250418):
    out = (C.c_uint8 * max(1, n))()
    lib().orc_synth(C.addressof(out), n, seed)
    return bytes(out[:n])


def random_bytes(n, seed):
    out = (C.c_uint8 * max(1, n))()
    lib().orc_random_bytes(C.addressof(out), n, seed)
    return bytes(out[:n])


ORC_GDEFLATE = 1


def make_params(chunk, mode="native", methods=(1, 3, 4, 255), prefs=None, n_total=None,
                exact_entropy=True, deflate="zlib"):
    """deflate: which id-5 encoder -- "zlib" (zlib.compress level 9, the
    reference's) or "gd" ("ambc-deflate v1", the GPU engine's)."""
    prefs = PREFS if prefs is None else prefs
    p = Params()
    p.chunk_size = chunk
    p.mode = 1 if mode == "reference" else 0
    p.flags = ORC_GDEFLATE if deflate == "gd" else 0
    mask = 0
    for m in methods:
        if m < 16:
            mask |= 1 << m
    p.method_mask = mask
    for mid in range(16):
        lo, hi = prefs.get(mid, (1, 0))
        p.pref_min[mid], p.pref_max[mid] = lo, min(hi, 0xFFFFFFFF)
    keep = []
    if exact_entropy:
        tf = entropy_table(chunk)
        keep.append(tf)
        p.ent_full = tf.ctypes.data
        if n_total is not None and n_total % chunk:
            tt = entropy_table(n_total % chunk)
            keep.append(tt)
            p.ent_tail = tt.ctypes.data
    p._keep = keep
    return p


def select(chunk_bytes, params, tab=None):
    src = _buf(chunk_bytes)
    pl = C.c_int64()
    t = tab if tab is not None else entropy_table(len(chunk_bytes))
    mid = lib().orc_select(C.addressof(src), len(chunk_bytes), C.byref(params), t.ctypes.data,
                           C.byref(pl))
    return mid, pl.value


def decide_all(data, params, nthreads=0):
    n = len(data)
    M = (n + params.chunk_size - 1) // params.chunk_size
    src = _buf(data)
    ids = (C.c_uint8 * max(1, M))()
    pl = (C.c_uint32 * max(1, M))()
    lib().orc_decide_all(C.addressof(src), n, C.byref(params), C.addressof(ids), C.addressof(pl),
                         nthreads)
    return list(ids[:M]), list(pl[:M])


def compress_body(data, params, nthreads=0):
    """_adaptive_compress restated: returns (body bytes, Stats)."""
    n = len(data)
    C_ = params.chunk_size
    M = (n + C_ - 1) // C_
    cap = n + 18 * M + 16 + 64 * M + 64
    src = _buf(data)
    out = (C.c_uint8 * cap)()
    st = Stats()
    r = lib().orc_compress_body(C.addressof(src), n, C.byref(params), C.addressof(out), cap,
                                C.byref(st), nthreads)
    if r == -2:
        raise struct.error("argument out of range")
    if r < 0:
        raise RuntimeError("oracle body overflow")
    return bytes(out[:r]), st


def np_entropy(d):
    """calculate_entropy (advanced_compression.py:48-57), numpy as the reference."""
    if not d:
        return 0.0
    counts = np.bincount(np.frombuffer(bytes(d), dtype=np.uint8), minlength=256)
    probs = counts / len(d)
    probs = probs[probs > 0]
    return -np.sum(probs * np.log2(probs))


def _lzma_xz(d):
    """LZMACompression.compress (advanced_compression.py:163-185)."""
    c = lzma.LZMACompressor(format=lzma.FORMAT_XZ, check=lzma.CHECK_CRC64,
                            filters=[{"id": lzma.FILTER_LZMA2, "dict_size": 1 << 24}])
    return c.compress(d) + c.flush()


_zstd = None


def zstd_lib():
    """The system libzstd (python-``zstandard``, the reference's id-8 library,
    is absent here).  None when it does not load."""
    global _zstd
    if _zstd is None:
        try:
            z = C.CDLL("libzstd.so.1")
        except OSError:
            return None
        z.ZSTD_getFrameContentSize.restype = C.c_ulonglong
        z.ZSTD_getFrameContentSize.argtypes = [C.c_char_p, C.c_size_t]
        z.ZSTD_findFrameCompressedSize.restype = C.c_size_t
        z.ZSTD_findFrameCompressedSize.argtypes = [C.c_char_p, C.c_size_t]
        z.ZSTD_decompress.restype = C.c_size_t
        z.ZSTD_decompress.argtypes = [C.c_void_p, C.c_size_t, C.c_char_p, C.c_size_t]
        z.ZSTD_compress.restype = C.c_size_t
        z.ZSTD_compress.argtypes = [C.c_void_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_int]
        z.ZSTD_compressBound.restype = C.c_size_t
        z.ZSTD_compressBound.argtypes = [C.c_size_t]
        z.ZSTD_isError.restype = C.c_uint
        z.ZSTD_isError.argtypes = [C.c_size_t]
        _zstd = z
    return _zstd


def zstd_compress(d, level=19):
    """ZstdCompressor(level=19).compress (advanced_compression.py:224-234): one
    frame carrying its content size."""
    z = zstd_lib()
    cap = z.ZSTD_compressBound(len(d))
    out = C.create_string_buffer(max(cap, 1))
    r = z.ZSTD_compress(out, cap, bytes(d), len(d), level)
    if z.ZSTD_isError(r):
        raise ValueError("zstd compress")
    return out.raw[:r]


def zstd_decompress(d, max_output_size):
    """ZstdDecompressor().decompress(d, max_output_size=...) of python-zstandard
    >= 0.15 (advanced_compression.py:240-241), restated on libzstd's one-shot
    API: the FIRST frame only (trailing bytes ignored), sized by its header's
    content size, or by max_output_size when the header has none; raises where
    python-zstandard raises ZstdError."""
    z = zstd_lib()
    d = bytes(d)
    cs = z.ZSTD_getFrameContentSize(d, len(d))
    if cs == (1 << 64) - 2:
        raise ValueError("error determining content size from frame header")
    if cs == 0:
        return b""
    unknown = cs == (1 << 64) - 1
    if unknown and max_output_size == 0:
        raise ValueError("could not determine content size in frame header")
    cap = max_output_size if unknown else cs
    flen = z.ZSTD_findFrameCompressedSize(d, len(d))
    if z.ZSTD_isError(flen):
        raise ValueError("did not decompress full frame")
    out = C.create_string_buffer(max(cap, 1))
    r = z.ZSTD_decompress(out, cap, d[:flen], flen)
    if z.ZSTD_isError(r) or (not unknown and r != cs):
        raise ValueError("decompression error")
    return out.raw[:r]


def select_reference_set(chunk, ids, prefs=None):
    """_pick_best_chunk_and_method's per-size method loop (adaptive_compressor.py:
    559-579) over the reference's stdlib set {1..7}: should_use, compress, keep the
    strict minimum of len + 18 in id order.  ids 1/2/3/5 through the C restatement,
    6/7 (bz2 / lzma) through the same stdlib calls as advanced_compression.py:112-213."""
    prefs = PREFS if prefs is None else prefs
    n = len(chunk)
    best, win, wl = n, 255, n
    for mid in sorted(i for i in ids if i != 255):
        lo, hi = prefs.get(mid, (1, 999999999))
        if not lo <= n <= hi:
            continue
        if mid in (1, 2, 3, 4, 5):
            if not should_use(mid, chunk):
                continue
            if mid == 4:
                continue                      # Delta: len == n never beats raw
            payload = {1: rle_encode, 2: dict_encode, 3: huff_encode, 5: deflate_encode}[mid](chunk)
            if payload is None:
                continue                      # Huffman raises on 1 or 256 symbols
        elif mid == 6:
            if n < 1024 or np_entropy(chunk) >= 7.7:
                continue
            payload = bz2.compress(chunk, compresslevel=9)
        elif mid == 7:
            if n < 8192 or np_entropy(chunk) >= 8.0:
                continue
            payload = _lzma_xz(chunk)
        elif mid == 8:
            if n < 512 or np_entropy(chunk) > 8.2:
                continue
            payload = zstd_compress(chunk)
        else:
            raise ValueError(mid)
        if len(payload) + 18 < best:
            best, win, wl = len(payload) + 18, mid, len(payload)
    return win, wl


def _encode_reference_set(mid, chunk):
    return {1: rle_encode, 2: dict_encode, 3: huff_encode, 5: deflate_encode,
            6: lambda d: bz2.compress(d, compresslevel=9), 7: _lzma_xz, 8: zstd_compress}[mid](chunk)


def compress_body_multisize(data, sizes, methods=(1, 3, 4, 255), prefs=None, deflate="gd",
                            reference_set=False):
    """_adaptive_compress with several CHUNK_SIZE_CANDIDATES
    (adaptive_compressor.py:363-394 with _pick_best_chunk_and_method :537-590):
    at every position each candidate size clamped to the remainder, its in-size
    winner by orc_select (ids ascending, strict '<'), sizes compared by the fp64
    ratio (len + 18) / size, strictly, in list order; a position where no size
    beats raw stores the remainder raw.  Returns (body, chunk_stats dict)."""
    n = len(data)
    enc = {1: rle_encode, 3: huff_encode, 9: lz4_frame_encode,
           5: gdeflate_encode if deflate == "gd" else deflate_encode}
    st = {"total_chunks": 0, "compressed_chunks": 0, "raw_chunks": 0,
          "method_usage": {m: 0 for m in methods}, "bytes_saved": 0, "original_size": n,
          "compressed_size_without_overhead": 0, "overhead_bytes": 0}
    out = bytearray()
    pos = 0
    while pos < n:
        remain = n - pos
        best = (1.0, remain, 255, 0)
        tried = {}
        for c in sizes:
            s = min(c, remain)
            if s <= 0:
                break
            if s not in tried:
                if reference_set:
                    tried[s] = select_reference_set(data[pos:pos + s], methods, prefs)
                else:
                    p = make_params(s, "native", methods, prefs, exact_entropy=False,
                                    deflate=deflate)
                    tried[s] = select(data[pos:pos + s], p, tab=entropy_table(s))
            mid, pl = tried[s]
            if mid != 255 and (pl + 18) / s < best[0]:
                best = ((pl + 18) / s, s, mid, pl)
        st["total_chunks"] += 1
        _, s, mid, pl = best
        if mid == 255:
            if remain > 0xFFFFFFFF:
                raise struct.error("argument out of range")
            out += MARKER + bytes((255, 0)) + struct.pack("<III", remain, remain, remain)
            out += data[pos:]
            st["raw_chunks"] += 1
            break
        chunk = data[pos:pos + s]
        payload = _encode_reference_set(mid, chunk) if reference_set else enc[mid](chunk)
        assert len(payload) == pl
        out += MARKER + bytes((mid, 0)) + struct.pack("<III", s, s, pl) + payload
        st["compressed_chunks"] += 1
        st["method_usage"][mid] += 1
        st["compressed_size_without_overhead"] += pl
        st["overhead_bytes"] += 18
        st["bytes_saved"] += s - (pl + 18)
        pos += s
    out += MARKER + bytes(12)
    st["overhead_bytes"] += 16
    return bytes(out), st


def build_header(data):
    """_build_header (adaptive_compressor.py:312-325) with the constant marker."""
    hdr = bytearray(b"AMBC")
    hdr.append(2)
    hdr += b"\x00\x00\x00\x00"
    hdr.append(32)
    hdr += MARKER
    hdr.append(1)
    hdr += hashlib.md5(data).digest()
    hdr += struct.pack("<Q", len(data))
    hdr += b"\x00" * 8
    hdr[5:9] = struct.pack("<I", len(hdr))
    return bytes(hdr)


def stats_dict(st, orig_size, comp_size, registered_ids, raw=False):
    """_calculate_compression_stats / _build_stats_raw (adaptive_compressor.py:257-284,482-520)."""
    if raw:
        return {"original_size": orig_size, "compressed_size": orig_size, "ratio": 1.0,
                "percent_reduction": 0.0, "overhead_bytes": 0, "compression_efficiency": 1.0,
                "chunk_stats": {"total_chunks": 1, "compressed_chunks": 0, "raw_chunks": 1,
                                "method_usage": {}, "bytes_saved": 0,
                                "original_size": orig_size,
                                "compressed_size_without_overhead": orig_size,
                                "overhead_bytes": 0}}
    usage = {str(m): int(st.method_usage[m]) for m in registered_ids}
    cs = {"total_chunks": int(st.total_chunks), "compressed_chunks": int(st.compressed_chunks),
          "raw_chunks": int(st.raw_chunks), "method_usage": usage,
          "bytes_saved": int(st.bytes_saved), "original_size": orig_size,
          "compressed_size_without_overhead": int(st.payload_bytes),
          "overhead_bytes": int(st.overhead_bytes)}
    if orig_size == 0:
        ratio, pr = 1.0, 0.0
    else:
        ratio = comp_size / orig_size
        pr = (1.0 - ratio) * 100.0
    if cs["compressed_chunks"] > 0:
        ocs = 0
        for mid in registered_ids:
            cnt = usage[str(mid)]
            if mid != 255 and cnt > 0:
                ocs += cnt / cs["total_chunks"] * orig_size
        eff = cs["compressed_size_without_overhead"] / ocs if ocs > 0 else 1.0
    else:
        eff = 1.0
    return {"original_size": orig_size, "compressed_size": comp_size, "ratio": ratio,
            "percent_reduction": pr, "chunk_stats": cs, "overhead_bytes": cs["overhead_bytes"],
            "compression_efficiency": eff}


def compress_file_bytes(data, chunk, mode="native", methods=(1, 3, 4, 255), nthreads=0):
    """AdaptiveCompressor.compress restated -> (file bytes, stats dict)."""
    p = make_params(chunk, mode, methods, n_total=len(data))
    body, st = compress_body(data, p, nthreads)
    hdr = build_header(data)
    if len(hdr) + len(body) > len(data):
        return bytes(data), stats_dict(st, len(data), len(data), methods, raw=True)
    hdr = hdr[:-8] + struct.pack("<Q", len(body))
    return hdr + body, stats_dict(st, len(data), len(hdr) + len(body), methods)


# ---------------------------------------------------------------------------
# decode side
# ---------------------------------------------------------------------------
def _c_dec(fn, payload, orig):
    out = (C.c_uint8 * max(1, orig + 256))()
    src = _buf(payload)
    r = getattr(lib(), fn)(C.addressof(src), len(payload), orig, C.addressof(out))
    return None if r < 0 else bytes(out[:r])


def _pad_trunc(b, orig):
    return b[:orig] if len(b) > orig else b + bytes(orig - len(b))


def decode_chunk(mid, payload, orig):
    """method.decompress(payload, orig) with the engine's except -> zeros (:437-442).
    Returns bytes, or None when ``mid`` has no registered method (verbatim copy)."""
    if mid == 255:                                  # NoCompression.decompress :691-713
        return _pad_trunc(payload, orig)
    if mid in (1, 2, 3, 4, 9):
        fn = {1: "orc_rle_decode", 2: "orc_dict_decode", 3: "orc_huff_decode",
              4: "orc_delta_decode", 9: "orc_lz4_frame_decode"}[mid]
        r = _c_dec(fn, payload, orig)
        return bytes(orig) if r is None else r
    if mid in (5, 6, 7, 8):
        if not payload:
            return b""
        try:
            raw = {5: zlib.decompress, 6: bz2.decompress, 7: lzma.decompress,
                   8: lambda b: zstd_decompress(b, orig)}[mid](payload)
            return _pad_trunc(raw, orig)
        except Exception:  # noqa: BLE001 -- reference wrappers return zeros
            return bytes(orig)
    return None


def decompress_body(body, orig_size, registered=(1, 2, 3, 4, 5, 6, 7, 9, 255),
                    return_produced=False):
    """_adaptive_decompress (adaptive_compressor.py:396-454).  With
    ``return_produced``: (output, bytes the packages produced before the final
    pad/truncate)."""
    out = bytearray()
    pos = 0
    n = len(body)
    while pos < n:
        if pos + 18 > n:
            break
        if body[pos:pos + 4] != MARKER:
            raise ValueError("Marker mismatch in chunk header.")
        t = body[pos + 4]
        _used, orig, clen = struct.unpack_from("<III", body, pos + 6)
        pos += 18
        if t == 0:
            break
        if pos + clen > n:
            break
        payload = body[pos:pos + clen]
        pos += clen
        r = decode_chunk(t, payload, orig) if t in registered else None
        out += payload if r is None else r
        if len(out) >= orig_size:
            break
    if return_produced:
        return _pad_trunc(bytes(out), orig_size), len(out)
    return _pad_trunc(bytes(out), orig_size)


def parse_header(blob):
    """_parse_header (adaptive_compressor.py:332-358)."""
    if blob[:4] != b"AMBC":
        raise ValueError("Magic mismatch")
    if blob[4] > 2:
        raise ValueError(f"Unsupported version: {blob[4]}")
    hsize = struct.unpack_from("<I", blob, 5)[0]
    mlen = blob[9]
    ms = (mlen + 7) // 8
    ctype = blob[10 + ms]
    csz = 16 if ctype == 1 else 0
    csum = blob[11 + ms:11 + ms + csz]
    op = 11 + ms + csz
    orig = struct.unpack_from("<Q", blob, op)[0]
    return {"header_size": hsize, "original_size": orig, "checksum": csum,
            "marker_bytes": blob[10:10 + ms]}


def decompress_file_bytes(blob, registered=(1, 2, 3, 4, 5, 6, 7, 9, 255)):
    h = parse_header(blob)
    out = decompress_body(blob[h["header_size"]:], h["original_size"], registered)
    if hashlib.md5(out).digest() != h["checksum"]:
        raise ValueError("Checksum mismatch => possibly corrupted file.")
    return out
