"""Huffman (id 3) package decoding on the GPU (k_decode_huff<4096|8192>, the
serial k_decode above 8 KiB) against the oracle's restatement of
HuffmanCompression.decompress (compression_methods.py:407-470) inside the
reference's _adaptive_decompress loop (adaptive_compressor.py:396-454).

Covers: payloads of the encoder for every kind of histogram (2..255 symbols,
text, skewed binary, one dominant byte), code lengths past the 10-bit lookup
(Fibonacci counts: codes of 17 bits from real data, 32-46 bits from crafted
tables), every orig rule (orig below, at and above the symbols, orig = 0 where
the reference still appends one symbol), nbits cut short / past the payload,
codes cut by the end of the bits, repeated table entries (last count wins, first
slot kept), zero counts, table errors (k entries past the payload, fewer than
two symbols), and the three routes (4 KiB / 8 KiB LDS kernels, serial kernel)
through both the host and the device header walk."""
import os
import struct

import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(hip_lib):
    from ambc import _lib
    return _lib.default_context()


def _pkg(t, orig, payload):
    return b"\xff\xff\x00\x00" + bytes((t, 0)) + struct.pack("<III", orig, orig, len(payload)) + payload


class _Env:
    def __init__(self, **kv):
        self.kv = {k: str(v) for k, v in kv.items()}

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update(self.kv)

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _decode_both(body, osz):
    """the GPU decode through the host walk and through the device walk"""
    from ambc import AdaptiveCompressor
    comp = AdaptiveCompressor()
    a = comp._adaptive_decompress(body, osz)
    with _Env(AMBC_DEVWALK_MIN=0, AMBC_WALK_PIECE=4096):
        b = comp._adaptive_decompress(body, osz)
    return a, b


def _check_packages(payloads_origs):
    """one body of type-3 packages; every package alone and the whole body"""
    body = b"".join(_pkg(3, o, p) for p, o in payloads_origs)
    for p, o in payloads_origs:
        single = _pkg(3, o, p)
        for osz in (max(o, 1), o + 3):
            want = orc.decompress_body(single, osz)
            a, b = _decode_both(single, osz)
            assert a == want, (len(p), o, osz)
            assert b == want, (len(p), o, osz)
    total = orc.decompress_body(body, 1 << 30, return_produced=True)[1]
    for osz in (total, total - 1, total + 17):
        want = orc.decompress_body(body, osz)
        a, b = _decode_both(body, osz)
        assert a == want and b == want, osz


def _fib_counts(n):
    f = [1, 1]
    while len(f) < n:
        f.append(f[-1] + f[-2])
    return f[:n]


def _skewed(rng, n, nsym, alpha):
    w = rng.pareto(alpha, nsym) + 1e-3
    syms = rng.choice(256, nsym, replace=False)
    return bytes(syms[rng.choice(nsym, n, p=w / w.sum())].astype(np.uint8))


def test_huffman_decode_encoder_payloads(ctx):
    rng = np.random.default_rng(61)
    cases = []
    words = [b"alpha", b"beta", b"gamma", b"delta", b"eps", b"zeta", b"eta", b"theta"]
    for n in (100, 257, 1000, 4096, 4095, 6000, 8192, 12000, 20000):
        text = b" ".join(words[i] for i in rng.integers(0, len(words), n // 4))[:n]
        cases.append(text)
        cases.append(_skewed(rng, n, int(rng.integers(2, 255)), 1.2))
        cases.append(_skewed(rng, n, 2, 3.0))
        d = bytearray(rng.integers(0, 2, n, dtype=np.uint8) * 7)
        d[0] = 200
        cases.append(bytes(d))                                         # one dominant byte
    # 255 distinct bytes with entropy < 7 (the widest table the encoder writes)
    d = bytearray(b"\x00" * 4000) + bytes(range(1, 255)) * 2
    cases.append(bytes(d))
    # Fibonacci counts: codes past the 10-bit lookup (17 bits at 18 symbols)
    f = _fib_counts(18)
    d = b"".join(bytes([i + 33]) * c for i, c in enumerate(f))[:8192]
    cases.append(bytes(rng.permutation(np.frombuffer(d, np.uint8))))
    pays = []
    for d in cases:
        p = orc.huff_encode(d)
        assert p is not None
        for o in (len(d), len(d) - 1 if len(d) > 1 else 1, len(d) // 3, 0, 1, len(d) + 9):
            pays.append((p, o))
    _check_packages(pays)


def _table(counts):
    return bytes([len(counts)]) + b"".join(bytes([s]) + struct.pack("<I", c) for s, c in counts)


def test_huffman_decode_crafted_payloads(ctx):
    rng = np.random.default_rng(62)
    pays = []
    # deep trees from the table alone (powers of two: depth 32; Fibonacci: depth 46), random bits
    for counts in ([(s, 1 << max(0, s - 1)) for s in range(33)],
                   [(200 - s, c) for s, c in enumerate(_fib_counts(47))]):
        for nbytes in (40, 600, 3000, 7000):
            bits = rng.integers(0, 256, nbytes, dtype=np.uint8).tobytes()
            for nb in (8 * nbytes, 8 * nbytes - 5, 8 * nbytes + 100, 3):
                pays.append((_table(counts) + struct.pack("<I", nb) + bits, 4096))
    good = orc.huff_encode(b"hello huffman world " * 100)
    k = good[0]
    tab_end = 1 + 5 * k
    bits = good[tab_end + 4:]
    nb = struct.unpack_from("<I", good, tab_end)[0]
    for cut in (0, 1, 3, len(bits) // 2, len(bits) - 1):          # the bits cut short
        pays.append((good[:tab_end + 4] + bits[:cut], 2000))
    for nbv in (0, 1, nb - 1, nb + 1, 1 << 31, 0xFFFFFFFF):        # nbits against the bytes
        pays.append((good[:tab_end] + struct.pack("<I", nbv) + bits, 2000))
    pays.append((good[:tab_end + 2], 2000))                        # nbits field cut
    pays.append((good[:tab_end], 2000))                            # no nbits field
    pays.append((good[:tab_end - 2], 2000))                        # last count cut (still parses)
    pays.append((good[:tab_end - 5], 2000))                        # last entry missing: IndexError
    pays.append((b"\x00" + struct.pack("<I", 99) + bits, 50))      # k = 0: heappop of []
    pays.append((_table([(65, 10)]) + struct.pack("<I", 40) + bits, 50))          # one symbol
    pays.append((_table([(65, 10), (65, 3)]) + struct.pack("<I", 40) + bits, 50))  # one distinct byte
    # repeated entries: the byte keeps its first slot, the last count wins
    dup = [(97, 5), (98, 5), (97, 1), (99, 2), (98, 9), (100, 0), (101, 0)]
    pays.append((_table(dup) + struct.pack("<I", 8 * len(bits)) + bits, 3000))
    # zero counts everywhere (ties broken by the byte)
    pays.append((_table([(s, 0) for s in (9, 3, 200, 1)]) + struct.pack("<I", 8 * len(bits)) + bits, 3000))
    # a 255-entry table with its bits, and one whose last entries lie past the payload
    t255 = _table([(s, int(rng.integers(1, 50))) for s in range(255)])
    pays.append((t255 + struct.pack("<I", 8 * len(bits)) + bits, 3000))
    pays.append((t255[:700], 3000))
    for o in (0, 1):
        pays.append((good, o))
    _check_packages(pays)


def test_huffman_decode_routes(ctx):
    """the same payloads through the 4 KiB / 8 KiB LDS kernels and the serial one
    (orig and clen around the route limits), in many-package bodies"""
    rng = np.random.default_rng(63)
    pays = []
    for n in (4090, 4096, 4097, 8191, 8192, 8193, 9000, 16384):
        d = _skewed(rng, n, 40, 1.5)
        p = orc.huff_encode(d)
        for o in (n, 4096, 4097, 8192, 8193, n + 100):
            pays.append((p, o))
    _check_packages(pays)
    # a body of many small and large packages, decoded through both walks
    parts, osz = [], 0
    for q in range(300):
        n = int(rng.integers(100, 9000))
        d = _skewed(rng, n, int(rng.integers(2, 120)), 1.0 + rng.random())
        p = orc.huff_encode(d)
        o = n if q % 7 else n + int(rng.integers(-50, 50))
        parts.append(_pkg(3, max(o, 0), p))
        osz += max(o, 0)
    body = b"".join(parts)
    want = orc.decompress_body(body, osz)
    a, b = _decode_both(body, osz)
    assert a == want and b == want


def test_huffman_plugin_orig_zero(ctx):
    """HuffmanCompression.decompress(payload, 0) appends one symbol before its
    length test (compression_methods.py:462-468); the other plugins give b''"""
    from ambc.methods import DeltaCompression, HuffmanCompression, NoCompression, RLECompression
    p = orc.huff_encode(b"abracadabra" * 20)
    assert HuffmanCompression().decompress(p, 0) == orc.decode_chunk(3, p, 0) == b"a"
    assert HuffmanCompression().decompress(p, 5) == orc.decode_chunk(3, p, 5)
    assert RLECompression().decompress(orc.rle_encode(b"\x05" * 40), 0) == orc.decode_chunk(1, orc.rle_encode(b"\x05" * 40), 0)
    assert DeltaCompression().decompress(b"\x01\x02", 0) == orc.decode_chunk(4, b"\x01\x02", 0)
    assert NoCompression().decompress(b"abc", 0) == b""
