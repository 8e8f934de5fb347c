"""id 5 as the reference computes it -- zlib.compress(data, 9)
(/root/reference/advanced_compression.py:76-81) -- on the GPU (ambc_zlib9.hip,
AMBC_FLAG_ZLIB9 / AdaptiveCompressor(deflate="zlib9")): whole bodies against the
oracle selector running the system zlib 1.2.11 for id 5, and every id-5 package
against Python's zlib.compress(chunk, 9), byte for byte."""
import random
import zlib

import pytest

from oracle import oracle as orc
from oracle import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(hip_lib):
    from ambc import _lib
    return _lib.default_context()


def _comp(**kw):
    from ambc import AdaptiveCompressor
    return AdaptiveCompressor(deflate="zlib9", **kw)


def _id5_packages(body, data):
    """(chunk bytes, payload) of every id-5 package of a native/reference body"""
    out = []
    pos = off = 0
    while pos + 18 <= len(body) and body[pos + 4] != 0:
        t = body[pos + 4]
        orig = int.from_bytes(body[pos + 10:pos + 14], "little")
        clen = int.from_bytes(body[pos + 14:pos + 18], "little")
        if t == 5:
            out.append((data[off:off + orig], body[pos + 18:pos + 18 + clen]))
        pos += 18 + clen
        off += orig
    return out


def _check(data, chunk, methods, modes=("native", "reference")):
    n = len(data)
    seen = 0
    for mode in modes:
        comp = _comp(chunk_size=chunk, mode=mode, methods=methods)
        body = comp._adaptive_compress(data)
        ref, st = orc.compress_body(data, orc.make_params(chunk, mode, methods, n_total=n, deflate="zlib"),
                                    nthreads=0)
        assert body == ref, (mode, n, chunk, methods)
        gst = comp._last_device_stats
        assert gst.method_usage[5] == st.method_usage[5]
        for raw, payload in _id5_packages(body, data):
            assert payload == zlib.compress(raw, 9)
            seen += 1
        assert comp._adaptive_decompress(body, n) == data
    return seen


Z9_CASES = [((1 << 20) + 77, 20250418, 4096, (1, 3, 4, 5, 9)), ((1 << 20) + 5, 3, 1024, (1, 3, 5)),
            (600001, 8, 4096, (5,)), (300000, 10, 2048, (3, 5, 9)), (250000, 12, 4096, (1, 2, 3, 4, 5)),
            (123457, 13, 1008, (5,)), (200000, 14, 4000, (1, 3, 4, 5)),
            # 8 KiB chunks: distances past TOO_FAR (4096), chains of 8192 positions
            (600000, 21, 8192, (1, 3, 4, 5, 9)), (300001, 22, 8192, (5,)), (250000, 23, 8192, (1, 2, 3, 4, 5)),
            (123456, 24, 6000, (1, 3, 5))]


@pytest.mark.parametrize("n,seed,chunk,methods", Z9_CASES)
def test_zlib9_bodies_match_zlib(ctx, n, seed, chunk, methods):
    assert _check(synth.generate(n, seed), chunk, methods) > 0


def test_zlib9_segmented_call_matches_zlib(ctx):
    """16385 chunks: the native call runs as pipelined segments, each segment's
    zlib-9 trees, emission and pending payloads on a second stream beside the next
    segment's encode and parse (ambc_host.cpp encode_range); body equal to the
    oracle's, every id-5 package equal to zlib.compress(chunk, 9)"""
    data = synth.generate((16 << 20) + 77, 31)
    assert _check(data, 1024, (1, 3, 4, 5), modes=("native",)) > 0


def _biased(n, p, seed):
    rng = random.Random(seed)
    return bytes(97 if rng.random() < p else 98 for _ in range(n))


def _alphabet(n, k, seed):
    """k random symbols: many length-3 matches, some only further back than TOO_FAR"""
    rng = random.Random(seed)
    sym = bytes(rng.sample(range(256), k))
    return bytes(rng.choice(sym) for _ in range(n))


def _words(n, seed, vocab=40):
    rng = random.Random(seed)
    ws = ["".join(rng.choice("etaoinshrdlu") for _ in range(rng.randint(1, 9))) for _ in range(vocab)]
    s = []
    while sum(map(len, s)) < n:
        s.append(rng.choice(ws) + rng.choice("  ,.\n"))
    return "".join(s).encode()[:n]


def test_zlib9_edge_chunks(ctx):
    """zero runs and 258-long matches, short periods (overlapping copies),
    biased binary data (hash chains past 1024 entries: the good_match chain cut
    after a >= 32 match), words from a small vocabulary (lazy matches), random
    bytes (stored blocks), tails below 64 bytes and odd lengths."""
    edge = [bytes(8192), b"ab" * 4096, b"abc" * 3000 + b"x", bytes(range(256)) * 32,
            b"\x07" * 5000 + bytes(range(256)) * 8, synth.random_bytes(12000, 4) + bytes(3000) + b"xyz" * 2000,
            b"q" * 4159, _biased(16384, 0.9, 1), _biased(16384, 0.97, 2), _biased(12288, 0.8, 3),
            _words(20000, 5), _words(16384, 6, vocab=6), synth.random_bytes(8193, 9),
            bytes(range(256)) * 4 + synth.random_bytes(3000, 10) + bytes(range(256)) * 4,
            _alphabet(16384, 24, 11), _alphabet(8192, 40, 12), _alphabet(12000, 64, 13)]
    seen = 0
    for d in edge:
        for chunk in (1024, 4096, 8192):
            seen += _check(d, chunk, (1, 3, 5, 9), modes=("native",))
    assert seen > 20


def test_zlib9_random_small_chunks(ctx):
    """many chunk contents from mixed generators at every size class"""
    rng = random.Random(77)
    parts = []
    for i in range(120):
        kind = rng.randrange(4)
        m = rng.randint(64, 4096)
        if kind == 0:
            parts.append(_words(m, i, vocab=rng.randint(3, 60)))
        elif kind == 1:
            parts.append(_biased(m, rng.choice((0.6, 0.9, 0.99)), i))
        elif kind == 2:
            parts.append(synth.generate(m, i))
        else:
            parts.append(bytes([rng.randrange(4)]) * rng.randint(1, 300) + _words(m, i, vocab=5))
    data = b"".join(parts)
    for chunk in (1024, 2048, 4096, 8192):
        assert _check(data, chunk, (5,), modes=("native",)) > 0


# chunks above 8 KiB (ambc_zlib9_big.hip): several blocks (a block per 16383
# symbols), distances up to MAX_DIST, the window slide past 65274 bytes
Z9_BIG_CASES = [((1 << 20) + 333, 31, 16384, (1, 3, 4, 5, 9)), ((1 << 20) + 5, 32, 32768, (5,)),
                ((1 << 20) + 17, 33, 65536, (1, 3, 4, 5)), (700001, 34, 65536, (5,)),
                (300000, 35, 12288, (1, 3, 5)), (400000, 36, 40000, (1, 2, 3, 4, 5))]


@pytest.mark.parametrize("n,seed,chunk,methods", Z9_BIG_CASES)
def test_zlib9_big_bodies_match_zlib(ctx, n, seed, chunk, methods):
    assert _check(synth.generate(n, seed), chunk, methods) > 0


def test_zlib9_big_edge_chunks(ctx):
    """64 KiB zero runs (258-splits over several windows), period-2 data, random
    bytes followed by zeros (stored blocks, then a Huffman block: the block split
    at 16383 symbols), small-vocabulary words and biased binary data (chains of
    4096 entries, MAX_DIST cuts), short alphabets (length-3 matches past
    TOO_FAR), and the window-slide inputs of tests/test_zlib9_model.py (a hash
    head of 32768 at step 65274 is NIL)."""
    from test_zlib9_model import slide_head_case
    edge = [bytes(65536), b"xy" * 32768, synth.random_bytes(40000, 41) + bytes(25536),
            synth.random_bytes(20000, 42) + _words(45536, 43), _words(65536, 44, vocab=12),
            _biased(65536, 0.93, 45), _alphabet(65536, 24, 46), _alphabet(50000, 90, 47),
            bytes(range(256)) * 256, synth.random_bytes(3000, 48) * 21 + b"!" * 1000]
    edge += [slide_head_case(n, n) for n in (65317, 65400, 65535)]
    seen = 0
    for d in edge:
        for chunk in (16384, 32768, 65536):
            seen += _check(d, chunk, (1, 3, 5), modes=("native",))
    assert seen > 20


def test_zlib9_big_random_chunk_contents(ctx):
    """chunk contents of every kind at 8193..65536 bytes (tails of odd length)"""
    rng = random.Random(78)
    parts = []
    for i in range(40):
        kind = rng.randrange(4)
        m = rng.randint(2000, 40000)
        if kind == 0:
            parts.append(_words(m, i, vocab=rng.randint(3, 200)))
        elif kind == 1:
            parts.append(_biased(m, rng.choice((0.6, 0.9, 0.99)), i))
        elif kind == 2:
            parts.append(synth.generate(m, i))
        else:
            parts.append(bytes([rng.randrange(4)]) * rng.randint(1, 3000) + _alphabet(m, rng.randint(3, 120), i))
    data = b"".join(parts)
    for chunk in (9008, 16384, 24576, 32768, 65536):
        assert _check(data, chunk, (5,), modes=("native",)) > 0


def _de_bruijn(k, n):
    """de Bruijn sequence B(k, n): every n-symbol string over k symbols exactly once"""
    a, seq = [0] * k * n, []

    def db(t, p):
        if t > n:
            if n % p == 0:
                seq.extend(a[1:p + 1])
        else:
            a[t] = a[t - p]
            db(t + 1, p)
            for j in range(a[t - p] + 1, k):
                a[t] = j
                db(t + 1, t)
    db(1, 1)
    return seq


def test_zlib9_no_repeat_chunks_decided_before_the_parse(ctx):
    """k_z9_parse decides chunks without a repeated 3-byte string from a lower
    bound of the all-literal block (round 6): bodies still equal the oracle with
    the system zlib, whether the bound loses (uniform random chunks) or not
    (repeat-free chunks over 16 symbols, which zlib-9 compresses by Huffman
    alone), and chunks with a single repeated string next to random bytes"""
    rng = random.Random(77)
    db16 = bytes(0x41 + x for x in _de_bruijn(16, 3))          # 4096 distinct 3-grams over 16 bytes
    parts = []
    for q in range(48):
        kind = q % 6
        if kind == 0:
            parts.append(bytes(rng.getrandbits(8) for _ in range(4096)))
        elif kind == 1:
            s = rng.randrange(0, len(db16))
            parts.append((db16 * 2)[s:s + 4096])
        elif kind == 2:
            b = bytearray(rng.getrandbits(8) for _ in range(4096))
            b[3000:3003] = b[100:103]                               # one 3-byte repeat
            parts.append(bytes(b))
        elif kind == 3:
            b = bytearray(rng.getrandbits(8) for _ in range(4096))
            b[4093:4096] = b[7:10]                                  # the repeat ends the chunk
            parts.append(bytes(b))
        elif kind == 4:
            parts.append(bytes(rng.choice(b"0123456789abcdef") for _ in range(4096)))   # many repeats
        else:
            parts.append(bytes(rng.getrandbits(7) for _ in range(4096)))                  # H0 ~ 7 bits
    data = b"".join(parts)
    for chunk, methods in ((4096, (1, 3, 4, 5)), (4096, (5,)), (2048, (1, 3, 5)), (8192, (1, 3, 4, 5, 9)),
                           (1024, (5,))):
        _check(data, chunk, methods)
