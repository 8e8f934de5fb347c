"""Drop-in AdaptiveCompressor for the MI355X path.

Same constructor, attributes, ``compress(input_file, output_file)`` /
``decompress(input_file, output_file)`` file API and stats dicts as the
reference (adaptive_compressor.py:49-700).  The two chunk loops
(``_adaptive_compress`` :363-394 with its selector :537-590, and
``_adaptive_decompress`` :396-454) are ONE C-ABI call each into
libambc_hip.so; the container header, MD5 and the whole-file raw fallback stay
here exactly as the reference writes them.

Chunking: the reference tries 8 candidate sizes at every position.  This
engine runs a single chunk size C (``chunk_size=``, default 4096), i.e.
``CHUNK_SIZE_CANDIDATES = [C]``, in one of two modes:

* ``mode='native'``    every C-byte chunk is decided independently (the
  reference's ``_pick_best_chunk_and_method(chunk, 0)`` + ``_process_chunk``
  per chunk);
* ``mode='reference'`` byte-identical to the reference loop with
  ``CHUNK_SIZE_CANDIDATES=[C]``, including its remainder-raw rule (the first
  chunk nothing compresses swallows the rest of the file as one raw chunk).

With several ``CHUNK_SIZE_CANDIDATES`` (e.g. the reference's default
``REFERENCE_CHUNK_SIZE_CANDIDATES``) the reference's multi-size walk runs
instead, on the device (``_adaptive_compress_multisize`` ->
ambc_compress_multisize_ex).  The reference's bz2 / LZMA codecs (ids 6 / 7) have no
GPU encoder: with them among ``methods`` (reference mode, or several candidates)
they are scored on host threads beside the device's encoders
(``hostcodecs.py``).

Defaults differ from the reference's ``AdaptiveCompressor()`` (8-candidate
walk, every stdlib codec): this class defaults to one 4096-byte chunk size,
native mode and methods {1, 3, 4, 9} (the throughput configuration; id 9 needs
an LZ4 decoder on the reading side).  The first compress of an instance built
with those defaults says so once (``DefaultsWarning``);
``AdaptiveCompressor.like_reference()`` builds the closest GPU configuration to
the reference's default instead (``full_set=True``: with bz2 / LZMA, byte for
byte the reference's default).
"""
import ctypes as C
import hashlib
import math
import os
import struct
import sys
import threading
import time
import warnings

import numpy as np

from . import _lib
from .container import (FORMAT_VERSION, MAGIC_NUMBER, MARKER_BYTES, MARKER_LENGTH,
                        build_header, marker_bytes_aligned, parse_header,
                        update_compressed_size)
from .methods import DECODE_METHODS, GPU_METHODS, NoCompression
from .registry import (DEFAULT_CHUNK_SIZE, DEFAULT_METHODS, HOST_LIBRARY_IDS, HOST_SCORED_IDS,
                       METHOD_CHUNK_PREFS, METHOD_NAMES, REFERENCE_CHUNK_SIZE_CANDIDATES, method_mask)

_TERMS = {}


def entropy_terms(n):
    """numpy's ``p * np.log2(p)`` for p = c/n, c = 0..n -- the exact terms
    HuffmanCompression.should_use sums (compression_methods.py:566-571).  The
    kernel only consults them when its fp64 entropy is within 1e-9 of 7.0."""
    t = _TERMS.get(n)
    if t is None:
        c = np.arange(n + 1, dtype=np.float64)
        p = c / float(n)
        with np.errstate(divide="ignore", invalid="ignore"):
            t = p * np.log2(p)
        t[0] = 0.0
        t = np.ascontiguousarray(t)
        if len(_TERMS) < 16:
            _TERMS[n] = t
    return t


class DefaultsWarning(UserWarning):
    """An instance with this engine's (not the reference's) encode defaults compresses."""


class AdaptiveCompressor:
    MAGIC_NUMBER = MAGIC_NUMBER
    FORMAT_VERSION = FORMAT_VERSION
    CHUNK_SIZE_CANDIDATES = [DEFAULT_CHUNK_SIZE]
    # the reference's default list (adaptive_compressor.py:61-62): set
    # CHUNK_SIZE_CANDIDATES to it for the reference's multi-size walk
    REFERENCE_CHUNK_SIZE_CANDIDATES = list(REFERENCE_CHUNK_SIZE_CANDIDATES)

    def __init__(self, marker_max_length=32, sample_size=10000, *, chunk_size=None,
                 mode="native", methods=None, devices=None, deflate=None):
        self.marker_max_length = marker_max_length
        self.sample_size = sample_size
        self.marker_finder = None          # the reference's finder is never called (:303-310)
        self.marker_bytes = None
        self.marker_length = 0
        self.marker_pattern = ""
        self.marker_bytes_aligned = b""
        self.marker_byte_length = 0
        self.use_multithreading = False
        self.max_workers = max(1, (os.cpu_count() or 2) - 1)
        self.progress_callback = None
        if mode not in ("native", "reference"):
            raise ValueError("mode must be 'native' or 'reference'")
        self.mode = mode
        # id 5's GPU encoder: "zlib9" (zlib.compress(data, 9)'s own bytes -- the
        # reference's DeflateCompression, advanced_compression.py:76-81) or "v1"
        # ("ambc-deflate v1": valid zlib streams of this engine's own parse,
        # faster); both take chunks up to the reference's 65536 prefs maximum.
        # None: "zlib9" in reference mode, else "v1".
        if deflate not in (None, "v1", "zlib9"):
            raise ValueError("deflate must be None, 'v1' or 'zlib9'")
        self._deflate = deflate
        # encode defaults left as they are: the first compress says they are not the reference's
        self._warn_defaults = chunk_size is None and mode == "native" and methods is None
        if chunk_size is not None:
            self.CHUNK_SIZE_CANDIDATES = [int(chunk_size)]
        ids = tuple(DEFAULT_METHODS if methods is None else [m for m in methods if m != 255])
        for i in ids:
            if i in HOST_SCORED_IDS and i not in DECODE_METHODS:
                raise ValueError(f"method id {i}: its host library is not available here")
        # validates: GPU encoders, plus the host-scored bz2 / lzma (ids 6 / 7)
        method_mask([i for i in ids if i not in HOST_SCORED_IDS])
        self.compression_methods = [(GPU_METHODS.get(i) or DECODE_METHODS[i])() for i in sorted(set(ids))]
        self.compression_methods.append(NoCompression())
        # decode side: every id the reference registers here (+ LZ4, which it
        # registers when python-lz4 is installed)
        self.method_lookup = {i: cls() for i, cls in DECODE_METHODS.items()}
        for m in self.compression_methods:
            self.method_lookup[m.type_id] = m
        self.method_names = dict(METHOD_NAMES)
        self.method_chunk_prefs = dict(METHOD_CHUNK_PREFS)
        self.devices = list(devices) if devices else None
        self.chunk_stats = None

    @classmethod
    def like_reference(cls, full_set=False, **kw):
        """The closest GPU configuration to the reference's ``AdaptiveCompressor()``
        (adaptive_compressor.py:61-62,64-178): its 8-candidate walk, reference mode,
        and its stdlib codecs that have GPU encoders -- RLE, Dictionary, Huffman,
        Delta and DEFLATE as zlib.compress(data, 9)'s own bytes at every size.
        full_set=True adds BZIP2 and LZMA (ids 6 / 7, no GPU encoder), scored on
        host threads beside the device's encoders: the reference's whole default
        method set, byte for byte (slow where the reference is: bz2 / lzma on
        every candidate chunk).  Without them, files where the reference would
        pick 6 / 7 differ; every package stays decodable by it."""
        ids = (1, 2, 3, 4, 5, 6, 7) if full_set else (1, 2, 3, 4, 5)
        comp = cls(mode="reference", methods=ids, **kw)
        comp.CHUNK_SIZE_CANDIDATES = list(REFERENCE_CHUNK_SIZE_CANDIDATES)
        return comp

    def _note_defaults(self):
        if self._warn_defaults and self.CHUNK_SIZE_CANDIDATES == [DEFAULT_CHUNK_SIZE]:
            self._warn_defaults = False
            warnings.warn("AdaptiveCompressor() defaults here are chunk_size=4096, mode='native', "
                          "methods (1, 3, 4, 9) -- not the reference's 8-candidate walk with its stdlib "
                          "codecs; id-9 (LZ4) packages need python-lz4 on the reading side.  Use "
                          "AdaptiveCompressor.like_reference() for the closest match, or methods=(1, 3, 4, 5) "
                          "for files a stdlib-only reference decodes",
                          DefaultsWarning, stacklevel=3)

    @property
    def deflate(self):
        if self._deflate is not None:
            return self._deflate
        if self.mode == "reference":
            return "zlib9"
        return "v1"

    # -- API parity helpers (adaptive_compressor.py:179-194) --------------------
    def set_progress_callback(self, callback):
        self.progress_callback = callback

    def _update_progress(self, stage, current, total, current_chunk=None, total_chunks=None):
        if self.progress_callback:
            self.progress_callback(stage, current, total, current_chunk, total_chunks)

    def enable_multithreading(self, max_workers=None):
        self.use_multithreading = True
        if max_workers:
            self.max_workers = max_workers
        print(f"Multithreading enabled with {self.max_workers} workers")

    def disable_multithreading(self):
        self.use_multithreading = False
        print("Multithreading disabled")

    def _init_marker(self, marker_bytes, marker_length):
        self.marker_bytes = marker_bytes
        self.marker_length = marker_length
        self.marker_pattern = "".join(format(b, "08b") for b in marker_bytes)[:marker_length]
        self.marker_bytes_aligned = marker_bytes_aligned(marker_bytes, marker_length)
        self.marker_byte_length = (marker_length + 7) // 8

    def _find_marker(self, file_data, sample_size):
        return MARKER_BYTES, MARKER_LENGTH

    # -- engine ------------------------------------------------------------------
    @property
    def chunk_size(self):
        cands = list(self.CHUNK_SIZE_CANDIDATES)
        if len(cands) != 1:
            raise ValueError("several CHUNK_SIZE_CANDIDATES: no single chunk size "
                             "(the multi-size walk runs in _adaptive_compress)")
        return int(cands[0])

    def _params(self, n):
        C_ = self.chunk_size
        p = _lib.Params()
        p.chunk_size = C_
        p.mode = _lib.MODE_REFERENCE if self.mode == "reference" else _lib.MODE_NATIVE
        p.flags = _lib.FLAG_ZLIB9 if self.deflate == "zlib9" else 0
        p.method_mask = method_mask(self._gpu_ids())
        for i in range(16):
            lo, hi = self.method_chunk_prefs.get(i, (1, 0))
            p.pref_min[i], p.pref_max[i] = max(0, lo), min(hi, 0xFFFFFFFF)
        keep = [entropy_terms(C_)]
        p.ent_full = keep[0].ctypes.data
        if n % C_:
            keep.append(entropy_terms(n % C_))
            p.ent_tail = keep[1].ctypes.data
        return p, keep

    def _ctx(self):
        return _lib.default_context(self.devices)

    def _gpu_ids(self):
        return [m.type_id for m in self.compression_methods
                if m.type_id != 255 and m.type_id not in HOST_SCORED_IDS]

    def _host_methods(self):
        return [m for m in self.compression_methods if m.type_id in HOST_SCORED_IDS]

    def _adaptive_compress_multisize(self, file_data):
        """_adaptive_compress (adaptive_compressor.py:363-394) with several
        CHUNK_SIZE_CANDIDATES: one C-ABI call, ambc_compress_multisize, runs the
        reference's walk (_pick_best_chunk_and_method :537-590: every candidate
        size clamped to the remainder, encoded as one chunk by the per-size method
        loop; sizes compared by their fp64 ratio, strictly, in list order; no
        winner -> the remainder raw) as many lock-step walks over the device-
        resident input, one batched encode per size and step."""
        n = len(file_data)
        ctx = self._ctx()
        cands = [int(c) for c in self.CHUNK_SIZE_CANDIDATES]
        p = _lib.Params()
        p.flags = _lib.FLAG_ZLIB9 if self.deflate == "zlib9" else 0
        p.method_mask = method_mask(self._gpu_ids())
        for i in range(16):
            lo, hi = self.method_chunk_prefs.get(i, (1, 0))
            p.pref_min[i], p.pref_max[i] = max(0, lo), min(hi, 0xFFFFFFFF)
        # numpy-exact entropy terms for every size Huffman may take on the walk:
        # the candidates and the remainders n - k*g (g = gcd: every position)
        lo3, hi3 = self.method_chunk_prefs.get(3, (1, 0))
        sizes = set()
        if 3 in self._gpu_ids():
            g = math.gcd(*cands)
            sizes = {c for c in cands if lo3 <= c <= hi3}
            k0, k1 = max(0, -(-(n - hi3) // g)), (n - lo3) // g if n >= lo3 else -1
            sizes |= {n - k * g for k in range(k0, k1 + 1)}
        tabs = [entropy_terms(sz) for sz in sorted(sizes)]
        ent_sizes = (C.c_uint32 * max(1, len(tabs)))(*sorted(sizes))
        ent_ptrs = (C.c_void_p * max(1, len(tabs)))(*[t.ctypes.data for t in tabs])
        carr = (C.c_uint32 * len(cands))(*cands)
        olen = C.c_uint64()
        st = _lib.Stats()
        src = file_data if isinstance(file_data, (bytes, bytearray)) else bytes(file_data)
        # ids 6 / 7: host-scored beside the device (hostcodecs.py)
        host = None
        if self._host_methods():
            from .hostcodecs import HostScorer
            host = HostScorer(src, self._host_methods(), self.method_chunk_prefs)
        # out = NULL: the body stays on the device until it is fetched into a
        # bytes object of exactly its size (see _adaptive_decompress for why
        # writing into a fresh, private bytes object is sound)
        with ctx.lock:                           # the device body below is the context's
            try:
                rc = ctx.lib.ambc_compress_multisize_ex(ctx.h, _lib.addr(src), n, C.byref(p), carr, len(cands),
                                                        ent_sizes, ent_ptrs, len(tabs),
                                                        C.addressof(host.struct) if host else None, None, 0,
                                                        C.byref(olen), C.byref(st))
            finally:
                if host:
                    host.close()
            if host and host.error is not None:
                raise host.error
            if rc == _lib.AMBC_E_RANGE:
                raise struct.error("argument out of range")
            if rc == _lib.AMBC_E_INVAL:
                raise NotImplementedError(_lib.last_error(ctx.lib))
            _lib.check(rc, ctx.lib)
            del tabs
            out = bytes(olen.value)
            if sys.getrefcount(out) != 2:
                raise RuntimeError("body buffer is shared: refusing to write into it")
            _lib.check(ctx.lib.ambc_fetch_body(ctx.h, C.cast(C.c_char_p(out), C.POINTER(C.c_uint8)),
                                               olen.value), ctx.lib)
        self._last_device_stats = st
        self.chunk_stats = {
            "total_chunks": int(st.total_chunks), "compressed_chunks": int(st.compressed_chunks),
            "raw_chunks": int(st.raw_chunks),
            "method_usage": {m.type_id: int(st.method_usage[m.type_id]) for m in self.compression_methods},
            "bytes_saved": int(st.bytes_saved), "original_size": n,
            "compressed_size_without_overhead": int(st.payload_bytes),
            "overhead_bytes": int(st.overhead_bytes)}
        self.method_usage_ids = [m.type_id for m in self.compression_methods]
        return out

    def _adaptive_compress(self, file_data):
        """One C-ABI call: input bytes -> .ambc body (packages + end chunk)."""
        self._note_defaults()
        if len(self.CHUNK_SIZE_CANDIDATES) != 1:
            return self._adaptive_compress_multisize(file_data)
        if self._host_methods():
            # host-scored ids: the reference loop with one candidate (reference mode)
            if self.mode != "reference":
                raise NotImplementedError("host-scored ids 6 / 7 (bz2 / lzma) need mode='reference' "
                                          "or several CHUNK_SIZE_CANDIDATES")
            return self._adaptive_compress_multisize(file_data)
        n = len(file_data)
        p, keep = self._params(n)
        ctx = self._ctx()
        cap = ctx.lib.ambc_compress_bound(n, p.chunk_size)
        out = bytearray(cap)
        olen = C.c_uint64()
        st = _lib.Stats()
        with ctx.lock:
            rc = ctx.lib.ambc_compress_batch(ctx.h, _lib.addr(file_data), n, C.byref(p),
                                             _lib.addr(out), cap, C.byref(olen), C.byref(st))
        if rc == _lib.AMBC_E_RANGE:
            import struct
            raise struct.error("argument out of range")
        _lib.check(rc, ctx.lib)
        del keep
        self._last_device_stats = st
        self.chunk_stats = {
            "total_chunks": int(st.total_chunks),
            "compressed_chunks": int(st.compressed_chunks),
            "raw_chunks": int(st.raw_chunks),
            "method_usage": {m.type_id: int(st.method_usage[m.type_id])
                             for m in self.compression_methods},
            "bytes_saved": int(st.bytes_saved),
            "original_size": n,
            "compressed_size_without_overhead": int(st.payload_bytes),
            "overhead_bytes": int(st.overhead_bytes),
        }
        self.method_usage_ids = [m.type_id for m in self.compression_methods]
        return bytes(memoryview(out)[:olen.value])

    def _adaptive_decompress(self, data, orig_size):
        """One C-ABI call: GPU kernels for ids 1/2/3/4/9/255 and unregistered ids,
        host zlib threads inside the library for id 5; ids 6/7 through the
        reference's library wrappers."""
        if self.marker_bytes_aligned not in (b"", MARKER_BYTES):
            raise NotImplementedError("only the reference's constant 32-bit marker is supported")
        ctx = self._ctx()
        data = bytes(data)
        # Large outputs: decode straight into a fresh (calloc'd, lazily zeroed)
        # bytes object -- this saves a full copy of the output (a second of CPU
        # per 4 GiB).  Writing into a bytes object is sound only while it is
        # private: created here, referenced by `out` alone, never hashed or
        # shared before the library has filled it.  The refcount check below
        # guards that invariant (2 = `out` + getrefcount's own argument).
        direct = orig_size >= (1 << 16)
        out = bytes(orig_size) if direct else bytearray(max(orig_size, 1))
        if direct and sys.getrefcount(out) != 2:
            raise RuntimeError("decode buffer is shared: refusing to write into it")
        reg = (C.c_uint64 * 4)()
        for t in self.method_lookup:
            reg[t >> 6] |= 1 << (t & 63)
        cap = 1 << 12
        while True:
            hc = (_lib.HostChunk * cap)()
            nh = C.c_uint32()
            st = _lib.Stats()
            optr = C.cast(C.c_char_p(out), C.POINTER(C.c_uint8)) if direct else _lib.addr(out)
            with ctx.lock:
                rc = ctx.lib.ambc_decompress_ex(ctx.h, _lib.addr(data), len(data), orig_size, reg,
                                                optr, hc, cap, C.byref(nh), C.byref(st))
            if rc == _lib.AMBC_E_CAPACITY and nh.value > cap:
                cap = nh.value
                continue
            if rc == _lib.AMBC_E_MARKER:
                raise ValueError("Marker mismatch in chunk header.")
            _lib.check(rc, ctx.lib)
            break
        if nh.value and direct:
            optr = C.cast(C.c_char_p(out), C.c_void_p).value
        for i in range(nh.value):                # ids 6/7: the reference's library wrappers
            h = hc[i]
            payload = data[h.body_off:h.body_off + h.clen]
            dec = self.method_lookup[h.type].decompress(payload, h.orig)
            end = min(h.out_off + len(dec), orig_size)
            if end > h.out_off:
                if direct:
                    C.memmove(optr + h.out_off, dec, end - h.out_off)
                else:
                    out[h.out_off:end] = dec[:end - h.out_off]
        self._last_device_stats = st
        return out if direct else bytes(memoryview(out)[:orig_size])

    # -- stats (adaptive_compressor.py:257-284,482-532) ---------------------------
    def _build_stats_raw(self, original_size, elapsed):
        tput = original_size / (1024 * 1024 * elapsed) if elapsed > 0 else 0.0
        chunk_stats = {"total_chunks": 1, "compressed_chunks": 0, "raw_chunks": 1,
                       "method_usage": {}, "bytes_saved": 0, "original_size": original_size,
                       "compressed_size_without_overhead": original_size, "overhead_bytes": 0}
        return {"original_size": original_size, "compressed_size": original_size, "ratio": 1.0,
                "percent_reduction": 0.0, "elapsed_time": elapsed,
                "throughput_mb_per_sec": tput, "chunk_stats": chunk_stats, "overhead_bytes": 0,
                "compression_efficiency": 1.0}

    def _calculate_compression_stats(self, orig_size, comp_size, elapsed):
        if orig_size == 0:
            ratio, pr = 1.0, 0.0
        else:
            ratio = comp_size / orig_size
            pr = (1.0 - ratio) * 100.0
        throughput = orig_size / (1024 * 1024 * elapsed) if elapsed > 0 else 0.0
        cs = self.chunk_stats
        if cs["compressed_chunks"] > 0:
            cdata = cs["compressed_size_without_overhead"]
            ocs = 0
            for mid, cnt in cs["method_usage"].items():
                if mid != 255 and cnt > 0:
                    ocs += cnt / cs["total_chunks"] * orig_size
            eff = cdata / ocs if ocs > 0 else 1.0
        else:
            eff = 1.0
        return {"original_size": orig_size, "compressed_size": comp_size, "ratio": ratio,
                "percent_reduction": pr, "elapsed_time": elapsed,
                "throughput_mb_per_sec": throughput, "chunk_stats": cs,
                "overhead_bytes": cs.get("overhead_bytes", 0),
                "compression_efficiency": eff}

    def _calculate_decompression_stats(self, csize, dsize, elapsed):
        tput = dsize / (1024 * 1024 * elapsed) if elapsed > 0 else 0.0
        return {"compressed_size": csize, "decompressed_size": dsize, "elapsed_time": elapsed,
                "throughput_mb_per_sec": tput}

    # -- file API (adaptive_compressor.py:221-301) ----------------------------------
    def compress_bytes(self, file_data):
        """compress() without the files: returns (container bytes, stats)."""
        start = time.time()
        marker_bytes, marker_len = self._find_marker(file_data, self.sample_size)
        self._init_marker(marker_bytes, marker_len)
        digest = {}
        th = threading.Thread(target=lambda: digest.setdefault("md5", hashlib.md5(file_data).digest()))
        th.start()                               # MD5 overlaps the device work
        try:
            body = self._adaptive_compress(file_data)
        finally:
            th.join()
        header = build_header(marker_bytes, marker_len, digest["md5"], len(file_data))
        final_size = len(header) + len(body)
        if final_size > len(file_data):
            print("Compression bigger than original => store raw.")
            return bytes(file_data), self._build_stats_raw(len(file_data), time.time() - start)
        header = update_compressed_size(header, len(body))
        return header + body, self._calculate_compression_stats(len(file_data), final_size,
                                                                 time.time() - start)

    def compress(self, input_file, output_file):
        start = time.time()
        with open(input_file, "rb") as f:
            file_data = f.read()
        blob, stats = self.compress_bytes(file_data)
        with open(output_file, "wb") as f:
            f.write(blob)
        stats["elapsed_time"] = time.time() - start
        if stats["elapsed_time"] > 0:
            stats["throughput_mb_per_sec"] = len(file_data) / (1024 * 1024 * stats["elapsed_time"])
        return stats

    def decompress_bytes(self, cdata):
        hdr = parse_header(cdata)
        self._init_marker(hdr["marker_bytes"], hdr["marker_length"])
        body = cdata[hdr["header_size"]:]
        out = self._adaptive_decompress(body, hdr["original_size"])
        if hashlib.md5(out).digest() != hdr["checksum"]:
            raise ValueError("Checksum mismatch => possibly corrupted file.")
        return out

    def decompress(self, input_file, output_file):
        start = time.time()
        with open(input_file, "rb") as f:
            cdata = f.read()
        hdr = parse_header(cdata)
        self._init_marker(hdr["marker_bytes"], hdr["marker_length"])
        body = cdata[hdr["header_size"]:]
        decompressed = self._adaptive_decompress(body, hdr["original_size"])
        with open(output_file, "wb") as f:
            f.write(decompressed)
        if hashlib.md5(decompressed).digest() != hdr["checksum"]:
            raise ValueError("Checksum mismatch => possibly corrupted file.")
        return self._calculate_decompression_stats(len(cdata), len(decompressed),
                                                   time.time() - start)


HOST_LIBRARY_IDS = HOST_LIBRARY_IDS
