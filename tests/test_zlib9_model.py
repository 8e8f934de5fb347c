"""oracle/zlib9_model.c -- the restatement of the reference's id-5 encoder,
zlib.compress(data, 9) (advanced_compression.py:76-81; zlib 1.2.11's deflate_slow
with its stored / static / dynamic block choice and heap-built trees) -- against
the system zlib the reference calls, byte for byte: chunk-sized inputs of every
class, 1..69 bytes, the 16383-symbol block split, 64 KiB, far 3-byte repeats
(TOO_FAR) and long chains (prev_length >= good_match)."""
import ctypes as C
import random
import zlib


from oracle import oracle as orc
from oracle import synth


def _z9(b):
    lib = orc.lib()
    f = lib.orc_zlib9
    f.argtypes = [C.c_char_p, C.c_uint32, C.c_void_p]
    f.restype = C.c_int64
    out = (C.c_uint8 * (len(b) + len(b) // 1000 + 64))()
    n = f(b, len(b), out)
    assert n > 0
    return bytes(out[:n])


def _gen(rnd, n):
    k = rnd.randrange(5)
    if k == 0:
        words = [bytes(rnd.choice(b"abcdefgh") for _ in range(rnd.randrange(2, 9))) for _ in range(rnd.randrange(2, 40))]
        return b" ".join(rnd.choice(words) for _ in range(n // 3 + 10))[:n]
    if k == 1:
        return b"".join(bytes([rnd.randrange(3)]) * rnd.randrange(1, 300) for _ in range(n))[:n]
    if k == 2:
        blk = bytes(rnd.randrange(256) for _ in range(rnd.randrange(20, 200)))
        s = bytearray((blk * (n // len(blk) + 1))[:n])
        for _ in range(rnd.randrange(0, 50)):
            s[rnd.randrange(n)] = rnd.randrange(256)
        return bytes(s)
    if k == 3:
        s = bytearray(rnd.randrange(256) for _ in range(n))
        for _ in range(n // 20):
            a, b = rnd.randrange(max(n - 3, 1)), rnd.randrange(max(n - 3, 1))
            s[b:b + 3] = s[a:a + 3]
        return bytes(s)
    return bytes(rnd.randrange(256) for _ in range(n))


def test_zlib9_model_matches_zlib():
    assert zlib.ZLIB_RUNTIME_VERSION == "1.2.11"
    rnd = random.Random(2026)
    mixed = synth.generate(1 << 20, 12)
    cases = [bytes(4096), b"ab" * 2048, bytes(range(256)) * 16, mixed[:4096]]
    cases += [_gen(rnd, n) for n in range(1, 70)]
    for _ in range(120):
        n = rnd.choice([64, 1000, 1024, 2048, 4096, 4096, 8192, 16384])
        o = rnd.randrange(0, len(mixed) - n)
        cases.append(mixed[o:o + n])
        cases.append(_gen(rnd, rnd.randrange(64, 16385)))
    cases += [_gen(rnd, n) for n in (16382, 16383, 16384, 16385, 65536)]
    cases += [bytes(rnd.randrange(256) for _ in range(n)) for n in (16383, 16384, 40000)]
    for c in cases:
        assert _z9(c) == zlib.compress(c, 9), len(c)


def _h15(b, p):
    return ((b[p] << 10) ^ (b[p + 1] << 5) ^ b[p + 2]) & 0x7FFF


def slide_head_case(seed, n, L=40):
    """Input where zlib's window slide decides a match: compressible bytes
    (0..127, geometric) with a 40-byte pattern of bytes >= 128 at 32768 and again
    at 65274, the slide step of an input shorter than 65536, and no position in
    between with the pattern's 15-bit hash -- so 65274's hash head is 32768,
    which the slid window reads as NIL (no match there; the copy is found one
    byte later, against 32769)."""
    rnd = random.Random(seed)
    while True:
        b = bytearray(min(int(rnd.expovariate(0.05)), 127) for _ in range(n))
        pat = bytes(rnd.randrange(128, 256) for _ in range(L))
        b[32768:32768 + L] = pat
        b[65274:65274 + L] = pat
        hh = _h15(b, 65274)
        if not any(_h15(b, p) == hh for p in range(32769, 65274)):
            return bytes(b)


def test_zlib9_model_window_slide():
    """8..64 KiB inputs (the reference's id-5 chunk sizes up to its 65536 prefs
    maximum, adaptive_compressor.py:119), the multi-block split there, and the
    window slide past 65274 bytes: the slide step's NIL head (inputs a model
    without the slide gets wrong) and sizes 65200..65536 of every class."""
    rnd = random.Random(65274)
    mixed = synth.generate(1 << 20, 13)
    cases = [slide_head_case(n, n) for n in (65317, 65400, 65535)]
    for n in (8193, 12288, 16384, 20000, 32767, 32768, 32769, 49152, 65273, 65274, 65275, 65276,
              65277, 65535, 65536):
        o = rnd.randrange(0, len(mixed) - n)
        cases += [mixed[o:o + n], _gen(rnd, n)]
    for _ in range(24):
        n = rnd.randrange(65200, 65537)
        cases.append(_gen(rnd, n))
        o = rnd.randrange(0, len(mixed) - n)
        cases.append(mixed[o:o + n])
    cases += [bytes(65536), b"xy" * 32768, bytes(range(256)) * 256]
    for c in cases:
        assert _z9(c) == zlib.compress(c, 9), len(c)
