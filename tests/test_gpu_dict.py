"""Dictionary (id 2) on the GPU (k_dict) vs the reference's own outputs and the
oracle restatement (oracle/ambc_oracle.c orc_dict_*, compression_methods.py:183-343).

- codec vectors: DictionaryCompression.compress / should_use against the bytes
  the reference produced (tests/golden/codecs.json);
- forced encodes of text, runs, periodic data (periods below and above the
  4096-byte window), random and mixed slices up to 8192 bytes: bit-exact with
  the oracle and round-tripping through the GPU decoder;
- whole bodies with id 2 among the candidates (native and reference modes,
  chunk sizes 1024 / 4096 / 8192 and ragged tails, with LZ4 and with DEFLATE):
  byte-identical to the oracle's selection, which keeps the reference's id order
  (ties go to the lower id)."""
import random

import pytest

from conftest import load_golden
from oracle import oracle as orc
from oracle import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(hip_lib):
    from ambc import _lib
    return _lib.default_context()


def test_dict_codec_vectors(ctx):
    from ambc.methods import DictionaryCompression
    m = DictionaryCompression()
    seen = 0
    for rec in load_golden("codecs.json"):
        d = bytes.fromhex(rec["data"])
        if len(d) > 8192 or "dictionary" not in rec:
            continue
        if rec["dictionary"]["ok"]:
            assert m.compress(d).hex() == rec["dictionary"]["out"], rec["name"]
            seen += 1
        assert m.should_use(d) == rec["should_use"]["2"], rec["name"]
    assert seen >= 20


def _cases():
    rnd = random.Random(4242)
    mixed = synth.generate(1 << 20, 31)
    text = ("This is a test text file with some repeating content. " * 200).encode()
    words = b" ".join(rnd.choice([b"the", b"of", b"and", b"GPU", b"chunk", b"wave", b"lane", b"x"])
                      for _ in range(3000))
    per5000 = bytes(rnd.randrange(256) for _ in range(5000))
    cases = [
        b"a", b"ab", b"abc", b"aaaa", bytes(100), bytes(4096), bytes(8192),
        b"A" * 1000 + b"B" * 1000 + b"C" * 1000,
        text[:4096], text[:8192], text[:1237], words[:8192], words[:4097], words[:5000],
        (per5000 + per5000)[:8192],                           # repeat beyond the window
        (per5000[:3000] * 3)[:8192],                          # repeat inside the window
        bytes(rnd.randrange(256) for _ in range(2048)),
        bytes(rnd.randrange(4) for _ in range(8192)),          # small alphabet, many short matches
        mixed[:4096], mixed[300000:308192], mixed[700001:704000], mixed[5:8197],
    ]
    for _ in range(6):
        n = rnd.randrange(1, 8193)
        o = rnd.randrange(0, len(mixed) - n)
        cases.append(mixed[o:o + n])
    return cases


def test_dict_forced_matches_oracle(ctx):
    from ambc.methods import DictionaryCompression
    m = DictionaryCompression()
    for d in _cases():
        enc = m.compress(d)
        assert enc == orc.dict_encode(d), len(d)
        assert m.decompress(enc, len(d)) == d, len(d)
        assert m.should_use(d) == orc.should_use(2, d), len(d)


def test_dict_encode_empty(ctx):
    from ambc.methods import DictionaryCompression
    assert DictionaryCompression().compress(b"") == b""
    assert DictionaryCompression(window_size=7, lookahead_size=-3).compress(b"") == b""


def _text_heavy(n, seed):
    """Mostly text and runs (where Dictionary can win), some random bytes."""
    rnd = random.Random(seed)
    vocab = [b"compress", b"the", b"adaptive", b"chunk", b"method", b"of", b"GPU", b"wave", b"\n"]
    out = bytearray()
    while len(out) < n:
        r = rnd.random()
        if r < 0.6:
            out += b" ".join(rnd.choice(vocab) for _ in range(rnd.randrange(20, 400)))
        elif r < 0.8:
            out += bytes([rnd.randrange(256)]) * rnd.randrange(10, 600)
        else:
            out += bytes(rnd.randrange(256) for _ in range(rnd.randrange(50, 900)))
    return bytes(out[:n])


BODY_CASES = [
    (200000, 1, 4096, (1, 2, 3, 4)),
    (150001, 2, 1024, (1, 2, 3, 4, 9)),
    (230000, 3, 8192, (1, 2, 3, 4)),
    (180000, 4, 8192, (1, 2, 3, 4, 9)),
    (120000, 5, 4096, (1, 2, 3, 4, 5)),
    (100003, 6, 2048, (2,)),
]


@pytest.mark.parametrize("n,seed,chunk,methods", BODY_CASES)
@pytest.mark.parametrize("mode", ["native", "reference"])
def test_dict_bodies_match_oracle(ctx, n, seed, chunk, methods, mode):
    from ambc import AdaptiveCompressor
    data = _text_heavy(n, seed) if seed % 2 else synth.generate(n, seed)
    comp = AdaptiveCompressor(chunk_size=chunk, mode=mode, methods=methods)
    body = comp._adaptive_compress(data)
    # id 5: reference mode writes zlib-9's own bytes (deflate=None)
    gd = 5 in methods and mode != "reference"
    ref, st = orc.compress_body(data, orc.make_params(chunk, mode, methods, n_total=n,
                                                      deflate="gd" if gd else "zlib"))
    assert len(body) == len(ref)
    assert body == ref
    assert comp.chunk_stats["method_usage"].get(2, 0) == st.method_usage[2]
    assert comp._adaptive_decompress(body, n) == data


@pytest.mark.parametrize("chunk", [4096, 8192])
def test_dict_walkers_at_scale(ctx, chunk):
    """The walker parse at scale (thousands of chunks, 64 walkers each): 8 MiB
    of mixed and text-heavy input with {1,2,3,4}, every body byte against the
    oracle's serial reference parse."""
    from ambc import AdaptiveCompressor
    for data in (synth.generate(8 << 20, 77), _text_heavy(8 << 20, 7)):
        comp = AdaptiveCompressor(chunk_size=chunk, methods=(1, 2, 3, 4))
        body = comp._adaptive_compress(data)
        ref, st = orc.compress_body(data, orc.make_params(chunk, "native", (1, 2, 3, 4), n_total=len(data)))
        assert body == ref
        assert st.method_usage[2] > 0


def test_dict_wins_and_ties(ctx):
    """Chunks where id 2 beats every other candidate, and the id-order tie rule."""
    from ambc import AdaptiveCompressor
    data = _text_heavy(300000, 9)
    comp = AdaptiveCompressor(chunk_size=4096, methods=(1, 2, 3, 4))
    body = comp._adaptive_compress(data)
    ref, st = orc.compress_body(data, orc.make_params(4096, "native", (1, 2, 3, 4), n_total=len(data)))
    assert body == ref
    assert st.method_usage[2] > 0


def _dict_tokens(rnd, n_tok, max_dist):
    """a random Dictionary token stream: literals, matches with any distance
    (0, beyond the output: Python negative indices, index errors) and length"""
    out = bytearray()
    for _ in range(n_tok):
        if rnd.random() < 0.5:
            out += bytes((0, rnd.randrange(256)))
        else:
            d = rnd.choice((0, 1, 2, 3, rnd.randrange(1, 64), rnd.randrange(1, max_dist)))
            out += bytes((rnd.randrange(1, 256), d & 255, d >> 8, rnd.choice((0, 1, 3, 40, 255, rnd.randrange(256)))))
    return bytes(out)


def test_dict_parallel_decode_lenient_streams(ctx):
    """dec_dict_par (k_decode_dict) against the oracle's restatement of
    DictionaryCompression.decompress (compression_methods.py:236-281) on crafted
    token streams: distances past the output start (negative indices, index
    errors -> zeros), distance 0 (repeat the last byte), tokens cut by the
    payload end, output reaching orig mid-window and mid-match, payloads that
    run out before orig (short packages: the host re-walk)."""
    import struct
    from ambc import AdaptiveCompressor
    rnd = random.Random(77)
    pk, orig_total = [], 0
    for k in range(400):
        toks = _dict_tokens(rnd, rnd.randrange(1, 700), rnd.choice((8, 300, 5000, 65535)))
        if k % 3 == 0:
            toks = toks[:rnd.randrange(1, len(toks) + 1)]          # cut anywhere
        if k % 5 == 0:                                             # valid prefix: literals first
            toks = bytes((0, 65)) * rnd.randrange(1, 40) + toks
        orig = rnd.choice((1, 7, 100, 1000, 4096, 4096, 8000, rnd.randrange(1, 8193)))
        pk.append(b"\xff\xff\x00\x00" + bytes((2, 0)) + struct.pack("<III", len(toks), orig, len(toks)) + toks)
        orig_total += orig
    body = b"".join(pk) + b"\xff\xff\x00\x00" + bytes(12)
    want = orc.decompress_body(body, orig_total)
    comp = AdaptiveCompressor(chunk_size=4096, methods=(1, 2, 3, 4))
    assert comp._adaptive_decompress(body, orig_total) == want
