"""ORACLE / TEST INFRASTRUCTURE ONLY -- never imported by the product path.

Pure-Python restatement of the reference's per-chunk compress loop, the CPU
baseline BASELINE.md §3.2 asks for ("the build's pure-Python CPU restatement,
timed on one core"): one C-byte chunk at a time, the reference's
``_pick_best_chunk_and_method(chunk, 0)`` (adaptive_compressor.py:537-590)
followed by ``_process_chunk`` (:631-700), with the codecs the reference runs
in Python:

* RLE      compress / should_use   compression_methods.py:78-114, 154-180
* Huffman  compress / should_use   compression_methods.py:354-405, 472-494, 551-574
* Delta    compress / should_use   compression_methods.py:585-608, 640-667

Byte loops stay byte loops (as in the reference), so its timing is the
reference's algorithm at CPython speed on this host.  Pinned by
tests/test_oracle.py: equal to the C oracle's body (itself pinned by the
reference-generated golden files) for the {1, 3, 4, 255} method set.
"""
import heapq
import struct

import numpy as np

MARKER = b"\xff\xff\x00\x00"
OVERHEAD = 18                       # _calculate_fixed_overhead (adaptive_compressor.py:623-629)
PREFS = {1: (32, 4096), 3: (32, 8192), 4: (32, 4096)}   # adaptive_compressor.py:114-127


def rle_compress(d):
    if not d:
        return b""
    out = bytearray()
    cur, cnt = d[0], 1
    for b in d[1:]:
        if b == cur and cnt < 255:
            cnt += 1
        else:
            out += bytes((cur, cnt))
            cur, cnt = b, 1
    out += bytes((cur, cnt))
    return bytes(out)


def _sampled(d, pred, bar):
    """RLE / Delta should_use: neighbours at a fixed step, ratio over (ss - 1)."""
    if len(d) < 4:
        return False
    ss = min(1000, len(d))
    step = max(1, len(d) // ss)
    hits = 0
    for i in range(0, len(d) - 1, step):
        if pred(d[i], d[i + 1]):
            hits += 1
    return hits / (ss - 1) > bar


def rle_should_use(d):
    return _sampled(d, lambda a, b: a == b, 0.3)


def delta_should_use(d):
    return _sampled(d, lambda a, b: abs(a - b) < 32, 0.5)


def delta_compress(d):
    if not d:
        return b""
    return bytes([d[0]] + [(d[i] - d[i - 1]) & 0xFF for i in range(1, len(d))])


def _first_order_counts(d):
    """symbol -> count in first-occurrence order (collections.Counter's order)."""
    counts = {}
    for b in d:
        counts[b] = counts.get(b, 0) + 1
    return counts


def huffman_should_use(d):
    if len(d) < 100:
        return False
    n = len(d)
    h = 0.0
    for c in _first_order_counts(d).values():
        p = c / n
        h -= p * np.log2(p)
    return h < 7.0


def huffman_compress(d):
    """Raises where the reference raises (1 or 256 distinct symbols)."""
    if not d:
        return b""
    counts = _first_order_counts(d)
    if len(counts) == 1:
        raise IndexError("string index out of range")       # code '' (compression_methods.py:527)
    # heap of (weight, first symbol, [symbols]); lo gets '0', hi gets '1'
    heap = [(w, s, [s]) for s, w in counts.items()]
    heapq.heapify(heap)
    code = {s: "" for s in counts}
    while len(heap) > 1:
        w0, f0, lo = heapq.heappop(heap)
        w1, _, hi = heapq.heappop(heap)
        for s in lo:
            code[s] = "0" + code[s]
        for s in hi:
            code[s] = "1" + code[s]
        heapq.heappush(heap, (w0 + w1, f0, lo + hi))
    out = bytearray((len(counts) & 0xFF,))
    if len(counts) > 255:
        raise ValueError("byte must be in range(0, 256)")   # compression_methods.py:382
    for s, c in counts.items():
        out.append(s)
        out += struct.pack("<I", c)
    bits = "".join(code[b] for b in d)
    out += struct.pack("<I", len(bits))
    for i in range(0, len(bits), 8):
        out.append(int(bits[i:i + 8].ljust(8, "0"), 2))
    return bytes(out)


CODECS = {1: (rle_should_use, rle_compress), 3: (huffman_should_use, huffman_compress),
          4: (delta_should_use, delta_compress)}


def package(chunk, methods=(1, 3, 4)):
    """One chunk's package: the in-size winner (strict <, list order) or raw."""
    n = len(chunk)
    best, best_id, best_data = 1.0, 255, None
    for mid in methods:
        lo, hi = PREFS[mid]
        if not lo <= n <= hi:
            continue
        use, enc = CODECS[mid]
        if use(chunk):
            try:
                c = enc(chunk)
            except (IndexError, ValueError):
                continue
            r = (len(c) + OVERHEAD) / n
            if r < best:
                best, best_id, best_data = r, mid, c
    if best_id != 255:
        best_data = CODECS[best_id][1](chunk)       # _process_chunk encodes the winner again
    if best_id == 255 or len(best_data) + OVERHEAD >= n:
        return MARKER + bytes((255, 0)) + struct.pack("<III", n, n, n) + bytes(chunk), 255
    return MARKER + bytes((best_id, 0)) + struct.pack("<III", n, n, len(best_data)) + best_data, best_id


def compress_body_native(data, chunk, methods=(1, 3, 4)):
    """Native mode: every chunk decided on its own; body incl. the 16-B end chunk."""
    out = bytearray()
    mv = memoryview(data)
    for p in range(0, len(data), chunk):
        pkg, _ = package(bytes(mv[p:p + chunk]), methods)
        out += pkg
    out += MARKER + bytes(12)
    return bytes(out)
